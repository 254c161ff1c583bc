// Native collective engine: Horovod's background loop (the reference
// runs it inside the Horovod core its image builds, horovod/Dockerfile:51-65, and every step's
// hvd.DistributedOptimizer allreduce at horovod/tensorflow_mnist.py:133 goes through it).
//
// One std::thread per process owns a framework RCCL communicator (rccl_comm.cpp) and a
// high-priority HIP stream from the PyTorch pool. Callers enqueue allreduces by name from any
// thread (autograd hooks included); the thread runs *cycles*:
//
//   1. drain the queue into per-slot FIFOs. A slot is a (name, dtype, numel, op) signature,
//      numbered in first-enqueue order on each rank.
//   2. negotiate with ONE small RCCL allreduce of a control vector (int32, summed over ranks):
//        [0] ranks asking to stop with nothing pending   [1] reserved (0)
//        [2 .. 2+S)       1 if this rank has work pending in slot s
//        [2+S .. 2+2S)    this rank's signature hash of slot s (0 if nothing pending)
//      Slot s is ready when its count equals the world size and the hash sum equals world x this
//      rank's hash (every rank enqueued the same signature there). Every rank sees the same
//      summed vector, so every rank derives the same ready list and issues the same RCCL calls
//      in the same order — the coordinator's role, as a bit-vector allreduce (Horovod's response
//      cache fast path) on the GPU instead of MPI messages to rank 0. A full count with a
//      mismatched hash is a signature error, reported on every rank.
//   3. fuse: ready slots in slot order, consecutive ones with equal dtype/op, packed into a
//      persistent device fusion buffer up to the threshold (one buffer, grown, never freed per
//      step) — copy-in / ncclAllReduce / copy-out on the engine stream; a tensor larger than the
//      threshold is reduced in place.
//   4. completion: each request's done event is recorded behind its copy-out and its handle
//      marked enqueued; wait() blocks the caller until then and makes the caller's current stream
//      wait for the event (no host-device sync on the caller's side).
//   5. stall inspector: a slot pending on some but not all ranks for warn_s is reported (with how
//      many ranks have it); after abort_s every pending handle fails and the process exits 134
//      so the launcher tears the job down (mpirun's semantics, horovod/tensorflow-mnist.yaml:17-38).
//
// Stream ordering: enqueue records an event on the caller's current stream (the producer of the
// gradient), the engine stream waits on it before reading; the tensor's storage is recorded on the
// engine stream so the caching allocator cannot hand it out before the engine is done with it.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mihvd {

// rccl_comm.cpp: the communicator behind a handle and the library's entry points
void* rccl_comm_raw(int64_t h);
int rccl_comm_world(int64_t h);
int rccl_comm_device(int64_t h);
int rccl_all_reduce_raw(void* buf, size_t count, int dtype, int op, void* comm, hipStream_t stream,
                        std::string* err);

namespace {

using Clock = std::chrono::steady_clock;

uint32_t fnv32(const std::string& s) {
  uint32_t h = 2166136261u;
  for (unsigned char c : s) h = (h ^ c) * 16777619u;
  return h == 0 ? 1u : h;  // 0 means "nothing pending"
}

int nccl_dtype(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "engine: unsupported dtype ", t);
  }
}

void hip_check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "engine: ", what, ": ", hipGetErrorString(e));
}

struct Handle {
  int state = 0;  // 0 queued, 1 enqueued on the engine stream, 2 failed
  hipEvent_t done = nullptr;
  std::string error;
  std::string name;
};

struct Req {
  int64_t id = 0;
  at::Tensor t;
  hipEvent_t ready = nullptr;
};

struct Slot {
  std::string name;
  uint32_t hash = 0;
  at::ScalarType dtype = at::kFloat;
  int op = 0;
  int64_t numel = 0;
  std::deque<Req> pending;
  Clock::time_point partial_since{};
  bool partial = false, warned = false;
};

}  // namespace

// Pure planning step, shared by the engine loop and the CPU unit test (engine_plan op): given the
// summed control vector, this rank's slot hashes and the slots' sizes/fuse keys, return the ready
// slots grouped for fusion (-1 separates groups), or throw on a signature mismatch.
std::vector<int64_t> engine_plan_groups(const int32_t* sum, int nslot, int world, const std::vector<uint32_t>& hash,
                                        const std::vector<int64_t>& bytes, const std::vector<int64_t>& key,
                                        int64_t threshold, std::vector<int>* partial, std::string* error) {
  std::vector<int64_t> out;
  int64_t cur_bytes = 0, cur_key = -1;
  bool open = false;
  for (int s = 0; s < nslot; ++s) {
    const int cnt = sum[2 + s];
    if (cnt == 0) continue;
    if (cnt < world) {
      if (partial) partial->push_back(s);
      continue;
    }
    const uint32_t hs = (uint32_t)sum[2 + nslot + s];
    if (hs != (uint32_t)((uint32_t)world * hash[s])) {
      if (error) *error = "slot " + std::to_string(s) + ": ranks enqueued different collectives (name/dtype/size/op)";
      return {};
    }
    const bool big = bytes[s] > threshold;
    if (open && (big || key[s] != cur_key || cur_bytes + bytes[s] > threshold)) {
      out.push_back(-1);
      open = false;
    }
    out.push_back(s);
    if (big) {
      out.push_back(-1);
      continue;
    }
    if (!open) {
      open = true;
      cur_bytes = 0;
      cur_key = key[s];
    }
    cur_bytes += bytes[s];
  }
  if (open) out.push_back(-1);
  return out;
}

namespace {

class Engine {
 public:
  Engine(int64_t comm, int64_t fusion_bytes, double cycle_s, double warn_s, double abort_s, int64_t max_slots)
      : comm_h_(comm),
        comm_(rccl_comm_raw(comm)),
        world_(rccl_comm_world(comm)),
        device_(rccl_comm_device(comm)),
        threshold_(fusion_bytes),
        cycle_(cycle_s),
        warn_s_(warn_s),
        abort_s_(abort_s),
        cap_((int)max_slots),
        stream_(c10::hip::getStreamFromPool(/*isHighPriority=*/true, (c10::DeviceIndex)device_)) {
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    auto i32 = at::TensorOptions().dtype(at::kInt);
    ctrl_dev_ = at::zeros({2 + 2 * (int64_t)cap_}, i32.device(at::kCUDA, device_));
    ctrl_host_ = at::zeros({2 + 2 * (int64_t)cap_}, i32.pinned_memory(true));
    thread_ = std::thread([this] { loop(); });
  }

  ~Engine() { stop(); }

  int64_t enqueue(const at::Tensor& t, const std::string& name, int64_t op) {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_ && t.is_contiguous(),
                "engine: expected a contiguous tensor on the engine's device ", device_);
    TORCH_CHECK(op >= 0 && op <= 3, "engine: op must be 0 sum, 1 prod, 2 max, 3 min");
    {
      std::lock_guard<std::mutex> lk(mu_);
      TORCH_CHECK(!stopping_, "engine: enqueue after stop");
      TORCH_CHECK(fatal_.empty(), "engine: the engine thread failed: ", fatal_);
    }
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    Req r;
    r.t = t;
    hip_check(hipEventCreateWithFlags(&r.ready, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventRecord(r.ready, c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream()), "hipEventRecord");
    auto h = std::make_shared<Handle>();
    h->name = name;
    hip_check(hipEventCreateWithFlags(&h->done, hipEventDisableTiming), "hipEventCreate");
    std::lock_guard<std::mutex> lk(mu_);
    TORCH_CHECK(!stopping_, "engine: enqueue after stop");
    TORCH_CHECK(fatal_.empty(), "engine: the engine thread failed: ", fatal_);
    r.id = next_id_++;
    handles_[r.id] = h;
    queue_.push_back({name, (int)op, std::move(r)});
    return queue_.back().req.id;
  }

  // Blocks until the collective of handle `id` is enqueued on the engine stream, then orders the
  // caller's current stream after it.
  void wait(int64_t id) {
    std::shared_ptr<Handle> h;
    {
      std::unique_lock<std::mutex> lk(mu_);
      auto it = handles_.find(id);
      TORCH_CHECK(it != handles_.end(), "engine: unknown or already waited handle ", id);
      h = it->second;
      cv_done_.wait(lk, [&] { return h->state != 0; });
      handles_.erase(it);
    }
    if (h->state == 2) {
      hipEventDestroy(h->done);
      TORCH_CHECK(false, "engine: collective '", h->name, "' failed: ", h->error);
    }
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    hip_check(hipStreamWaitEvent(c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream(), h->done, 0),
              "hipStreamWaitEvent");
    hipEventDestroy(h->done);
  }

  // true once the collective has completed on the device
  bool poll(int64_t id) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = handles_.find(id);
    TORCH_CHECK(it != handles_.end(), "engine: unknown handle ", id);
    if (it->second->state == 0) return false;
    if (it->second->state == 2) return true;
    return hipEventQuery(it->second->done) == hipSuccess;
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stopping_) return;
      stopping_ = true;
    }
    if (thread_.joinable()) thread_.join();
  }

  std::vector<int64_t> stats() {
    std::lock_guard<std::mutex> lk(mu_);
    return {cycles_, collectives_, tensors_, fused_bytes_, (int64_t)slots_.size(), stalls_warned_};
  }

 private:
  struct Item {
    std::string name;
    int op;
    Req req;
  };

  void fail_all(const std::string& why) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& kv : handles_)
      if (kv.second->state == 0) {
        kv.second->state = 2;
        kv.second->error = why;
      }
    fatal_ = why;
    cv_done_.notify_all();
  }

  int slot_of(const Item& it) {
    const std::string sig = it.name + "|" + std::to_string((int)it.req.t.scalar_type()) + "|" +
                            std::to_string(it.req.t.numel()) + "|" + std::to_string(it.op);
    auto f = slot_index_.find(sig);
    if (f != slot_index_.end()) return f->second;
    TORCH_CHECK((int)slots_.size() < cap_, "engine: more than ", cap_, " distinct collectives (MIHVD_ENGINE_SLOTS)");
    Slot s;
    s.name = it.name;
    s.hash = fnv32(sig);
    s.dtype = it.req.t.scalar_type();
    s.op = it.op;
    s.numel = it.req.t.numel();
    slots_.push_back(std::move(s));
    slot_index_[sig] = (int)slots_.size() - 1;
    return (int)slots_.size() - 1;
  }

  void loop() {
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    hipStream_t st = stream_.stream();
    auto next = Clock::now();
    bool stop_seen = false;
    try {
      while (!stop_seen) {
        // a world with nothing pending anywhere for 100 cycles backs off to 10x the cycle time
        // (every rank sees the same summed vectors, so all back off together); work ends it
        next += std::chrono::microseconds((int64_t)(cycle_ * 1e6 * (idle_ > 100 ? 10 : 1)));
        std::this_thread::sleep_until(next);
        if (Clock::now() > next + std::chrono::milliseconds(50)) next = Clock::now();
        bool stopping;
        {
          std::lock_guard<std::mutex> lk(mu_);
          while (!queue_.empty()) {
            Item it = std::move(queue_.front());
            queue_.pop_front();
            const int s = slot_of(it);
            slots_[s].pending.push_back(std::move(it.req));
          }
          stopping = stopping_;
        }
        // 2. negotiation: one small allreduce of the control vector
        int32_t* hv = ctrl_host_.data_ptr<int32_t>();
        const int S = cap_;
        std::fill(hv, hv + 2 + 2 * S, 0);
        bool any_pending = false;
        for (size_t s = 0; s < slots_.size(); ++s)
          if (!slots_[s].pending.empty()) {
            hv[2 + s] = 1;
            hv[2 + S + s] = (int32_t)slots_[s].hash;
            any_pending = true;
          }
        // a stopping rank first drains its own pending work (its peers will match it)
        hv[0] = (stopping && !any_pending) ? 1 : 0;
        hip_check(hipMemcpyAsync(ctrl_dev_.data_ptr(), hv, (2 + 2 * S) * 4, hipMemcpyHostToDevice, st), "H2D");
        std::string err;
        if (rccl_all_reduce_raw(ctrl_dev_.data_ptr(), 2 + 2 * S, ncclInt32, ncclSum, comm_, st, &err) != 0)
          throw std::runtime_error("negotiation allreduce: " + err);
        hip_check(hipMemcpyAsync(hv, ctrl_dev_.data_ptr(), (2 + 2 * S) * 4, hipMemcpyDeviceToHost, st), "D2H");
        hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
        {
          std::lock_guard<std::mutex> lk(mu_);
          ++cycles_;
        }
        if (hv[0] == world_) stop_seen = true;  // every rank asked to stop with nothing pending
        bool idle = true;
        for (int s = 0; s < S && idle; ++s) idle = hv[2 + s] == 0;
        idle_ = idle ? idle_ + 1 : 0;
        // 3. plan + execute
        std::vector<uint32_t> hash(S, 0);
        std::vector<int64_t> bytes(S, 0), key(S, 0);
        for (size_t s = 0; s < slots_.size(); ++s) {
          hash[s] = slots_[s].hash;
          bytes[s] = slots_[s].numel * (int64_t)c10::elementSize(slots_[s].dtype);
          key[s] = (int64_t)slots_[s].dtype * 16 + slots_[s].op;
        }
        std::vector<int> partial;
        std::string perr;
        const auto plan = engine_plan_groups(hv, S, world_, hash, bytes, key, threshold_, &partial, &perr);
        if (!perr.empty()) throw std::runtime_error(perr);
        std::vector<int> group;
        for (int64_t e : plan) {
          if (e >= 0) {
            group.push_back((int)e);
            continue;
          }
          run_group(group, st);
          group.clear();
        }
        inspect_stalls(partial);
      }
    } catch (const std::exception& e) {
      fail_all(e.what());
      std::fprintf(stderr, "[mihvd engine] fatal: %s\n", e.what());
      return;
    }
    fail_all("engine stopped");
  }

  void run_group(const std::vector<int>& group, hipStream_t st) {
    std::vector<Req> reqs;
    for (int s : group) {
      reqs.push_back(std::move(slots_[s].pending.front()));
      slots_[s].pending.pop_front();
      slots_[s].partial = slots_[s].warned = false;
    }
    for (auto& r : reqs) {
      hip_check(hipStreamWaitEvent(st, r.ready, 0), "hipStreamWaitEvent");
      c10::hip::HIPCachingAllocator::recordStream(r.t.storage().data_ptr(), stream_);
    }
    const Slot& s0 = slots_[group[0]];
    const int dt = nccl_dtype(s0.dtype);
    const ncclRedOp_t op = (ncclRedOp_t)s0.op;  // 0 sum, 1 prod, 2 max, 3 min == ncclRedOp_t
    std::string err;
    int64_t total = 0;
    if (reqs.size() == 1) {
      total = reqs[0].t.numel();
      if (rccl_all_reduce_raw(reqs[0].t.data_ptr(), (size_t)total, dt, op, comm_, st, &err) != 0)
        throw std::runtime_error("allreduce " + s0.name + ": " + err);
    } else {
      const int64_t es = (int64_t)c10::elementSize(s0.dtype);
      int64_t nbytes = 0;
      for (auto& r : reqs) nbytes += r.t.numel() * es;
      if (!fusion_.defined() || fusion_.numel() < nbytes) {
        // grown, never shrunk; the old buffer's last use is on this stream
        fusion_ = at::empty({std::max<int64_t>(nbytes, threshold_)}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, device_));
      }
      char* base = (char*)fusion_.data_ptr();
      int64_t off = 0;
      for (auto& r : reqs) {
        const int64_t nb = r.t.numel() * es;
        hip_check(hipMemcpyAsync(base + off, r.t.data_ptr(), nb, hipMemcpyDeviceToDevice, st), "copy-in");
        off += nb;
      }
      total = nbytes / es;
      if (rccl_all_reduce_raw(base, (size_t)total, dt, op, comm_, st, &err) != 0)
        throw std::runtime_error("fused allreduce: " + err);
      off = 0;
      for (auto& r : reqs) {
        const int64_t nb = r.t.numel() * es;
        hip_check(hipMemcpyAsync(r.t.data_ptr(), base + off, nb, hipMemcpyDeviceToDevice, st), "copy-out");
        off += nb;
      }
    }
    std::lock_guard<std::mutex> lk(mu_);
    ++collectives_;
    tensors_ += (int64_t)reqs.size();
    if (reqs.size() > 1) fused_bytes_ += total * (int64_t)c10::elementSize(s0.dtype);
    for (auto& r : reqs) {
      auto it = handles_.find(r.id);
      if (it != handles_.end()) {
        hip_check(hipEventRecord(it->second->done, st), "hipEventRecord");
        it->second->state = 1;
      }
      hipEventDestroy(r.ready);
    }
    cv_done_.notify_all();
  }

  void inspect_stalls(const std::vector<int>& partial) {
    const auto now = Clock::now();
    std::vector<char> is_partial(slots_.size(), 0);
    for (int s : partial) {
      is_partial[s] = 1;
      Slot& sl = slots_[s];
      if (!sl.partial) {
        sl.partial = true;
        sl.partial_since = now;
        continue;
      }
      const double age = std::chrono::duration<double>(now - sl.partial_since).count();
      if (warn_s_ > 0 && age > warn_s_ && !sl.warned) {
        sl.warned = true;
        const int have = ctrl_host_.data_ptr<int32_t>()[2 + s];
        std::fprintf(stderr,
                     "[mihvd engine] stall: '%s' has been submitted by %d of %d ranks for %.1f s (the others "
                     "have not reached it)\n",
                     sl.name.c_str(), have, world_, age);
        std::lock_guard<std::mutex> lk(mu_);
        ++stalls_warned_;
      }
      if (abort_s_ > 0 && age > abort_s_) {
        std::fprintf(stderr, "[mihvd engine] stall on '%s' exceeded %.1f s: aborting (exit 134)\n", sl.name.c_str(),
                     abort_s_);
        std::fflush(stderr);
        std::_Exit(134);
      }
    }
    for (size_t s = 0; s < slots_.size(); ++s)
      if (!is_partial[s]) slots_[s].partial = slots_[s].warned = false;
  }

  const int64_t comm_h_;
  void* comm_;
  const int world_, device_;
  const int64_t threshold_;
  const double cycle_, warn_s_, abort_s_;
  const int cap_;
  c10::hip::HIPStream stream_;
  at::Tensor ctrl_dev_, ctrl_host_, fusion_;
  std::vector<Slot> slots_;
  std::unordered_map<std::string, int> slot_index_;
  std::mutex mu_;
  std::condition_variable cv_done_;
  std::deque<Item> queue_;
  std::map<int64_t, std::shared_ptr<Handle>> handles_;
  int64_t next_id_ = 1;
  bool stopping_ = false;
  std::string fatal_;
  int64_t idle_ = 0;
  int64_t cycles_ = 0, collectives_ = 0, tensors_ = 0, fused_bytes_ = 0, stalls_warned_ = 0;
  std::thread thread_;
};

std::mutex g_emu;
std::unique_ptr<Engine> g_engine;

Engine& engine() {
  std::lock_guard<std::mutex> lk(g_emu);
  TORCH_CHECK(g_engine != nullptr, "engine: not started (engine_start)");
  return *g_engine;
}

}  // namespace

void engine_start(int64_t comm, int64_t fusion_bytes, double cycle_s, double warn_s, double abort_s,
                  int64_t max_slots) {
  TORCH_CHECK(fusion_bytes > 0 && cycle_s > 0 && max_slots > 0, "engine_start: bad arguments");
  std::lock_guard<std::mutex> lk(g_emu);
  TORCH_CHECK(g_engine == nullptr, "engine_start: an engine is already running");
  g_engine = std::make_unique<Engine>(comm, fusion_bytes, cycle_s, warn_s, abort_s, max_slots);
}

int64_t engine_allreduce_async(const at::Tensor& t, const std::string& name, int64_t op) {
  return engine().enqueue(t, name, op);
}

void engine_wait(int64_t h) { engine().wait(h); }

bool engine_poll(int64_t h) { return engine().poll(h); }

std::vector<int64_t> engine_stats() { return engine().stats(); }

void engine_stop() {
  std::unique_ptr<Engine> e;
  {
    std::lock_guard<std::mutex> lk(g_emu);
    e = std::move(g_engine);
  }
  if (e) e->stop();
}

bool engine_running() {
  std::lock_guard<std::mutex> lk(g_emu);
  return g_engine != nullptr;
}

// CPU-testable planning step: `ctrl` is a summed control vector (int32 [2 + 2 S]), `hash` this
// rank's slot hashes (int64, low 32 bits), `bytes` / `key` per slot. Returns the grouped ready
// slots (-1 ends a group), -2 followed by the partial slots; throws on a signature mismatch.
std::vector<int64_t> engine_plan(const at::Tensor& ctrl, int64_t world, const at::Tensor& hash, const at::Tensor& bytes,
                                 const at::Tensor& key, int64_t threshold) {
  const int S = (int)hash.numel();
  auto c = ctrl.to(at::kInt).contiguous();
  TORCH_CHECK(c.numel() == 2 + 2 * S, "engine_plan: ctrl must hold 2 + 2 S entries");
  auto hh = hash.to(at::kLong).contiguous(), bb = bytes.to(at::kLong).contiguous(), kk = key.to(at::kLong).contiguous();
  std::vector<uint32_t> hv(S);
  std::vector<int64_t> bv(S), kv(S);
  for (int s = 0; s < S; ++s) {
    hv[s] = (uint32_t)hh.data_ptr<int64_t>()[s];
    bv[s] = bb.data_ptr<int64_t>()[s];
    kv[s] = kk.data_ptr<int64_t>()[s];
  }
  std::vector<int> partial;
  std::string err;
  auto out = engine_plan_groups(c.data_ptr<int32_t>(), S, (int)world, hv, bv, kv, threshold, &partial, &err);
  TORCH_CHECK(err.empty(), "engine_plan: ", err);
  out.push_back(-2);
  for (int s : partial) out.push_back(s);
  return out;
}

int64_t engine_signature_hash(const std::string& sig) { return (int64_t)fnv32(sig); }

}  // namespace mihvd

TORCH_LIBRARY_FRAGMENT(mihvd, m) {
  m.def("engine_start(int comm, int fusion_bytes, float cycle_s, float warn_s, float abort_s, int max_slots) -> ()",
        &mihvd::engine_start);
  m.def("engine_allreduce_async(Tensor(a!) t, str name, int op=0) -> int", &mihvd::engine_allreduce_async);
  m.def("engine_wait(int handle) -> ()", &mihvd::engine_wait);
  m.def("engine_poll(int handle) -> bool", &mihvd::engine_poll);
  m.def("engine_stats() -> int[]", &mihvd::engine_stats);
  m.def("engine_stop() -> ()", &mihvd::engine_stop);
  m.def("engine_running() -> bool", &mihvd::engine_running);
  m.def("engine_plan(Tensor ctrl, int world, Tensor hash, Tensor bytes, Tensor key, int threshold) -> int[]",
        &mihvd::engine_plan);
  m.def("engine_signature_hash(str sig) -> int", &mihvd::engine_signature_hash);
}
