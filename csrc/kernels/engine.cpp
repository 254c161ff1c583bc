// Native collective engine: Horovod's background loop (the reference
// runs it inside the Horovod core its image builds, horovod/Dockerfile:51-65, and every step's
// hvd.DistributedOptimizer allreduce at horovod/tensorflow_mnist.py:133 goes through it).
//
// One std::thread per process owns two framework RCCL communicators (rccl_comm.cpp): a CONTROL
// communicator for negotiation on a control stream, and a DATA communicator for the fused
// allreduces on a high-priority data stream. Callers enqueue allreduces by name from any thread
// (autograd hooks included). The thread is event-driven: it sleeps on a condition variable while
// this rank has nothing pending and wakes on enqueue (no fixed clock); while work is pending it runs
// *cycles* back to back, or re-negotiates after at most the cycle time when its last cycle made no
// progress (MIHVD_CYCLE_TIME is a bound on that re-poll, not a floor on latency):
//
//   1. drain the queue. A signature (name, dtype, numel, op) gets a SLOT that every rank agrees
//      on: slots are keyed by the signature's 32-bit hash and numbered in an order all ranks derive
//      from the same data (see 3), never in a rank's local enqueue order — so ranks may enqueue
//      tensors in different orders.
//   2. negotiate with ONE small RCCL allreduce of a control vector (int32, summed over ranks) on
//      the control communicator:
//        [0] ranks asking to stop with nothing pending   [1] ranks with unannounced signatures
//        [2 .. 2+S)       1 if this rank has work pending in slot s
//        [2+S .. 2+2S)    the slot's hash if pending here (0 otherwise)
//      Slot s is ready when its count equals the world size (and the hash sum equals world x hash,
//      a consistency check). Every rank sees the same summed vector, derives the same ready list and
//      issues the same RCCL calls in the same order — the coordinator's role as a bit-vector
//      allreduce (Horovod's response-cache fast path) on the GPU instead of MPI messages to rank 0.
//   3. new signatures (only when [1] > 0): an all-gather of up to K unannounced hashes per rank;
//      every rank takes the union of the hashes that have no slot yet, sorts it and appends it to
//      the slot table (engine_new_slot_order) — identical on every rank by construction. A slot
//      table overflow is detected identically on every rank.
//   4. fuse: ready slots in slot order, consecutive ones with equal dtype/op, packed into a
//      persistent device fusion buffer up to the threshold by ONE batched pack kernel, one
//      ncclAllReduce, ONE batched unpack kernel — on the data stream. The host does not wait for
//      them: the next cycle's negotiation (control stream) overlaps them.
//   5. completion: each request's done event (from a pool) is recorded behind its unpack and its
//      handle marked enqueued; wait() blocks the caller until then and makes the caller's current
//      stream wait for the event (no host-device sync on the caller's side).
//   6. stall inspector: a slot pending on some but not all ranks for warn_s is reported (with how
//      many ranks have it), and so is a negotiation that peers have not joined for warn_s; after
//      abort_s the process exits 134 so the launcher tears the job down (mpirun's semantics,
//      horovod/tensorflow-mnist.yaml:17-38).
//
// Failures: an error every rank sees identically (a signature mismatch, the slot table overflowing)
// fails every pending handle on every rank and stops the engine. A failure local to one rank (a HIP
// or RCCL error) aborts both communicators and exits 134: its peers would otherwise wait forever in
// the next negotiation, where no stall inspector of theirs can tell them why.
//
// Stream ordering: enqueue records an event on the caller's current stream (the producer of the
// gradient); the data stream waits on it before reading; the tensor's storage is recorded on the data
// stream so the caching allocator cannot hand it out before the engine is done with it. The fusion
// buffer is allocated on the data stream (its only user); a replaced buffer is freed stream-ordered.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../runtime/slot_agreement.h"

namespace mihvd {

// rccl_comm.cpp: the communicator behind a handle and the library's entry points
void* rccl_comm_raw(int64_t h);
int rccl_comm_world(int64_t h);
int rccl_comm_device(int64_t h);
int rccl_all_reduce_raw(void* buf, size_t count, int dtype, int op, void* comm, hipStream_t stream,
                        std::string* err);
int rccl_all_gather_raw(const void* in, void* out, size_t count, int dtype, void* comm, hipStream_t stream,
                        std::string* err);
void rccl_comm_abort_raw(void* comm);

// ------------------------------------------------------------------------------------------------
// batched pack / unpack: one launch copies up to kCopyMax (src, dst, bytes) pieces; blockIdx.y is
// the piece, blockIdx.x strides over its bytes with the widest access its alignment allows
// ------------------------------------------------------------------------------------------------
constexpr int kCopyMax = 32;
struct CopyBatch {
  const char* src[kCopyMax];
  char* dst[kCopyMax];
  int64_t bytes[kCopyMax];
};

template <typename V>
__device__ __forceinline__ void copy_span(const char* s, char* d, int64_t nbytes) {
  const int64_t n = nbytes / (int64_t)sizeof(V);
  const V* sv = reinterpret_cast<const V*>(s);
  V* dv = reinterpret_cast<V*>(d);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dv[i] = sv[i];
}

__global__ void __launch_bounds__(256) engine_batched_copy_kernel(CopyBatch b) {
  const int k = blockIdx.y;
  const char* s = b.src[k];
  char* d = b.dst[k];
  const int64_t nb = b.bytes[k];
  const uintptr_t a = (uintptr_t)s | (uintptr_t)d | (uintptr_t)nb;
  if ((a & 15) == 0) copy_span<uint4>(s, d, nb);
  else if ((a & 7) == 0) copy_span<uint2>(s, d, nb);
  else if ((a & 3) == 0) copy_span<uint32_t>(s, d, nb);
  else if ((a & 1) == 0) copy_span<uint16_t>(s, d, nb);
  else copy_span<uint8_t>(s, d, nb);
}

namespace {

using Clock = std::chrono::steady_clock;

uint32_t fnv32(const std::string& s) { return engine_fnv32(s); }  // 0 is reserved: "nothing pending"

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

// a failure every rank sees identically (computed from the same summed / gathered data)
struct ConsistentError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("engine: ") + what + ": " + hipGetErrorString(e));
}

struct Handle {
  int state = 0;  // 0 queued, 1 enqueued on the data stream, 2 failed
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
  uint32_t hash = 0;
  bool known = false;  // dtype/op/numel/name set (from a local enqueue of this signature)
  std::string name;
  at::ScalarType dtype = at::kFloat;
  int op = 0;
  int64_t numel = 0;
  std::deque<Req> pending;
  Clock::time_point partial_since{};
  bool partial = false, warned = false;
};

}  // namespace

// engine_plan_groups / engine_new_slot_order and the slot table itself (SlotAgreement) live in
// csrc/runtime/slot_agreement.h: the same code runs over the TCP store in the CPU tests.

namespace {

constexpr int kAnnounce = 64;  // new signatures announced per rank per cycle

class Engine {
 public:
  Engine(int64_t comm, int64_t ctrl_comm, int64_t fusion_bytes, double cycle_s, double warn_s, double abort_s,
         int64_t max_slots)
      : comm_(rccl_comm_raw(comm)),
        ctrl_comm_(rccl_comm_raw(ctrl_comm)),
        world_(rccl_comm_world(comm)),
        device_(rccl_comm_device(comm)),
        threshold_(fusion_bytes),
        cycle_(cycle_s),
        warn_s_(warn_s),
        abort_s_(abort_s),
        cap_((int)max_slots),
        stream_(c10::hip::getStreamFromPool(/*isHighPriority=*/true, (c10::DeviceIndex)device_)),
        ctrl_stream_(c10::hip::getStreamFromPool(/*isHighPriority=*/true, (c10::DeviceIndex)device_)),
        agree_(world_, (int)max_slots, kAnnounce) {
    TORCH_CHECK(rccl_comm_world(ctrl_comm) == world_ && rccl_comm_device(ctrl_comm) == device_,
                "engine: the control communicator must span the same ranks and device");
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    auto i32 = at::TensorOptions().dtype(at::kInt);
    const int64_t n = 2 + 2 * (int64_t)cap_;
    ctrl_dev_ = at::zeros({n}, i32.device(at::kCUDA, device_));
    ctrl_host_ = at::zeros({n}, i32.pinned_memory(true));
    ann_dev_ = at::zeros({(int64_t)world_ * kAnnounce + kAnnounce}, i32.device(at::kCUDA, device_));
    ann_host_ = at::zeros({(int64_t)world_ * kAnnounce + kAnnounce}, i32.pinned_memory(true));
    hip_check(hipEventCreateWithFlags(&ctrl_ev_, hipEventDisableTiming), "hipEventCreate");
    hip_check(hipEventCreateWithFlags(&data_ev_, hipEventDisableTiming), "hipEventCreate");
    ctrl_.e = this;
    thread_ = std::thread([this] { loop(); });
  }

  ~Engine() {
    stop();
    for (hipEvent_t e : pool_) hipEventDestroy(e);
    if (ctrl_ev_) hipEventDestroy(ctrl_ev_);
    if (data_ev_) hipEventDestroy(data_ev_);
  }

  int64_t enqueue(const at::Tensor& t, const std::string& name, int64_t op) {
    TORCH_CHECK(t.is_cuda() && t.get_device() == device_ && t.is_contiguous(),
                "engine: expected a contiguous tensor on the engine's device ", device_);
    TORCH_CHECK(op >= 0 && op <= 3, "engine: op must be 0 sum, 1 prod, 2 max, 3 min");
    (void)nccl_dtype(t.scalar_type());
    const std::string sig =
        name + "|" + std::to_string((int)t.scalar_type()) + "|" + std::to_string(t.numel()) + "|" + std::to_string(op);
    const uint32_t h = fnv32(sig);
    {
      std::lock_guard<std::mutex> lk(mu_);
      TORCH_CHECK(!stopping_, "engine: enqueue after stop");
      TORCH_CHECK(fatal_.empty(), "engine: the engine thread failed: ", fatal_);
      auto it = local_sig_.find(h);
      if (it == local_sig_.end()) {
        // the slot cap, checked where the caller can see it (a new signature this rank adds)
        TORCH_CHECK((int)local_sig_.size() < cap_, "engine: more than ", cap_,
                    " distinct collectives (MIHVD_ENGINE_SLOTS)");
        local_sig_.emplace(h, sig);
      } else {
        TORCH_CHECK(it->second == sig, "engine: signature hash collision between '", it->second, "' and '", sig, "'");
      }
    }
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    Req r;
    r.t = t;
    r.ready = event_get();
    hip_check(hipEventRecord(r.ready, c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream()),
              "hipEventRecord");
    auto hd = std::make_shared<Handle>();
    hd->name = name;
    hd->done = event_get();
    int64_t id = 0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stopping_ || !fatal_.empty()) {
        event_put(r.ready);
        event_put(hd->done);
        TORCH_CHECK(false, "engine: enqueue after stop", fatal_.empty() ? "" : ": ", fatal_);
      }
      id = next_id_++;
      r.id = id;
      handles_[id] = hd;
      queue_.push_back({name, (int)op, h, std::move(r)});
      ++enqueued_;
    }
    cv_work_.notify_one();
    return id;
  }

  // Blocks until the collective of handle `id` is enqueued on the data stream, then orders the
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
      event_put(h->done);
      TORCH_CHECK(false, "engine: collective '", h->name, "' failed: ", h->error);
    }
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    const hipError_t e =
        hipStreamWaitEvent(c10::hip::getCurrentHIPStream((c10::DeviceIndex)device_).stream(), h->done, 0);
    // the wait captured the event's current record: re-recording it later (pool reuse) is safe
    event_put(h->done);
    TORCH_CHECK(e == hipSuccess, "engine: hipStreamWaitEvent: ", hipGetErrorString(e));
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

  // (called by one owner: engine_stop moves the engine out of the global first)
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stopping_ = true;
    }
    cv_work_.notify_all();
    if (thread_.joinable()) thread_.join();
  }

  std::vector<int64_t> stats() {
    std::lock_guard<std::mutex> lk(mu_);
    return {cycles_, collectives_, tensors_, fused_bytes_, (int64_t)slots_.size(), stalls_warned_, wakeups_,
            idle_waits_, announces_};
  }

 private:
  struct Item {
    std::string name;
    int op;
    uint32_t hash;
    Req req;
  };

  hipEvent_t event_get() {
    {
      std::lock_guard<std::mutex> lk(pool_mu_);
      if (!pool_.empty()) {
        hipEvent_t e = pool_.back();
        pool_.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }

  void event_put(hipEvent_t e) {
    if (e == nullptr) return;
    std::lock_guard<std::mutex> lk(pool_mu_);
    pool_.push_back(e);
  }

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

  bool local_work() const {
    if (!unassigned_.empty()) return true;
    for (const auto& s : slots_)
      if (!s.pending.empty()) return true;
    return false;
  }

  Slot& slot_for_local(int s, const Item& it) {
    Slot& sl = slots_[s];
    if (!sl.known) {
      sl.known = true;
      sl.name = it.name;
      sl.dtype = it.req.t.scalar_type();
      sl.op = it.op;
      sl.numel = it.req.t.numel();
    }
    return sl;
  }

  // the queue -> slot FIFOs (assigned signatures) or the unassigned staging area
  void drain_locked() {
    while (!queue_.empty()) {
      Item it = std::move(queue_.front());
      queue_.pop_front();
      const int s = agree_.slot(it.hash);
      if (s >= 0) {
        slot_for_local(s, it).pending.push_back(std::move(it.req));
        continue;
      }
      agree_.want(it.hash);  // announced in the coming cycles
      unassigned_[it.hash].push_back(std::move(it));
    }
  }

  // Polls `ev` (control stream) until it completes; meanwhile runs the negotiation stall check.
  // `quiet`: a rank that is stopping with nothing pending waits for its peers to finish their work
  // (they may be busy for long, e.g. rank 0 checkpointing) -- a clean wait, not a stall, so no
  // warning; but a peer that died during shutdown must not hold it forever: the abort still
  // fires, at twice the stall-abort time.
  void wait_ctrl(hipEvent_t ev, bool quiet = false) {
    const auto t0 = Clock::now();
    bool warned = false;
    int spins = 0;
    for (;;) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) hip_check(q, "negotiation event");
      if (++spins > 64) std::this_thread::sleep_for(std::chrono::microseconds(spins > 4096 ? 200 : 10));
      if ((spins & 255) != 0) continue;
      const double age = std::chrono::duration<double>(Clock::now() - t0).count();
      const double abort_after = quiet ? 2.0 * abort_s_ : abort_s_;
      if (!quiet && warn_s_ > 0 && age > warn_s_ && !warned) {
        warned = true;
        std::string names;
        for (const auto& s : slots_)
          if (!s.pending.empty()) names += (names.empty() ? "" : ", ") + s.name;
        for (const auto& kv : unassigned_)
          if (!kv.second.empty()) names += (names.empty() ? "" : ", ") + kv.second.front().name;
        std::fprintf(stderr,
                     "[mihvd engine] stall: this rank has waited %.1f s in negotiation for peers that have not "
                     "submitted any collective (pending here: %s)\n",
                     age, names.empty() ? "nothing" : names.c_str());
        std::lock_guard<std::mutex> lk(mu_);
        ++stalls_warned_;
      }
      if (abort_s_ > 0 && age > abort_after) {
        std::fprintf(stderr, "[mihvd engine] negotiation stalled for more than %.1f s%s: aborting (exit 134)\n",
                     abort_after, quiet ? " while stopping" : "");
        std::fflush(stderr);
        std::_Exit(134);
      }
    }
  }

  void loop() {
    c10::hip::HIPGuard g((c10::DeviceIndex)device_);
    // the data stream is this thread's current stream: the fusion buffer is allocated on it
    c10::hip::HIPStreamGuard sg(stream_);
    hipStream_t cst = ctrl_stream_.stream();
    bool progressed = true;
    try {
      for (;;) {
        bool stopping;
        {
          std::unique_lock<std::mutex> lk(mu_);
          const bool had_work = local_work();
          if (!had_work && queue_.empty() && !stopping_) {
            // idle: sleep until work or stop (no clock)
            ++idle_waits_;
            cv_work_.wait(lk, [&] { return !queue_.empty() || stopping_; });
            ++wakeups_;
          } else if (had_work && !progressed && queue_.empty() && !stopping_) {
            // partial work and no progress last cycle: re-negotiate within the cycle time, sooner
            // on new work
            cv_work_.wait_for(lk, std::chrono::microseconds((int64_t)(cycle_ * 1e6)),
                              [&] { return !queue_.empty() || stopping_; });
          }
          drain_locked();
          stopping = stopping_;
        }
        // 2. negotiation on the control communicator (slot_agreement.h)
        const int S = cap_;
        std::vector<int> pending;
        bool any_pending = !unassigned_.empty();
        for (size_t s = 0; s < slots_.size(); ++s)
          if (!slots_[s].pending.empty()) {
            pending.push_back((int)s);
            any_pending = true;
          }
        // a stopping rank first drains its own pending work (its peers will match it)
        ctrl_.quiet = stopping && !any_pending;
        const std::vector<int32_t> summed = agree_.negotiate(ctrl_, pending, stopping && !any_pending);
        const int32_t* hv = summed.data();
        std::copy(summed.begin(), summed.end(), ctrl_host_.data_ptr<int32_t>());  // (the stall report's view)
        {
          std::lock_guard<std::mutex> lk(mu_);
          ++cycles_;
        }
        if (hv[0] == world_) break;  // every rank asked to stop with nothing pending
        progressed = false;
        // 3. new signatures: all-gather the announced hashes, append their sorted union
        if (hv[1] > 0) {
          announce_round();
          progressed = true;
        }
        // 4. plan + execute on the data stream
        std::vector<uint32_t> hash(S, 0);
        std::vector<int64_t> bytes(S, 0), key(S, 0);
        for (size_t s = 0; s < slots_.size(); ++s) {
          hash[s] = slots_[s].hash;
          if (slots_[s].known) {
            bytes[s] = slots_[s].numel * (int64_t)c10::elementSize(slots_[s].dtype);
            key[s] = (int64_t)slots_[s].dtype * 16 + slots_[s].op;
          }
        }
        std::vector<int> partial;
        std::string perr;
        const auto plan = engine_plan_groups(hv, S, world_, hash, bytes, key, threshold_, &partial, &perr);
        if (!perr.empty()) throw ConsistentError(perr);
        std::vector<int> group;
        for (int64_t e : plan) {
          if (e >= 0) {
            group.push_back((int)e);
            continue;
          }
          run_group(group);
          group.clear();
          progressed = true;
        }
        inspect_stalls(partial);
      }
    } catch (const ConsistentError& e) {
      fail_all(e.what());
      std::fprintf(stderr, "[mihvd engine] fatal (on every rank): %s\n", e.what());
      return;
    } catch (const std::exception& e) {
      // local failure: the peers are (or will be) blocked in a collective with this rank
      fail_all(e.what());
      std::fprintf(stderr, "[mihvd engine] fatal on this rank: %s; aborting the engine communicators (exit 134)\n",
                   e.what());
      std::fflush(stderr);
      rccl_comm_abort_raw(ctrl_comm_);
      rccl_comm_abort_raw(comm_);
      std::_Exit(134);
    }
    fail_all("engine stopped");
  }

  // The control plane's collectives on the control communicator: staged through small device
  // buffers on the control stream, which first waits for the data stream's last collective (the
  // control communicator's kernels never run beside the data communicator's: two communicators
  // whose kernels overlap in different orders on different ranks can deadlock).
  struct RcclCtrl final : CtrlTransport {
    Engine* e = nullptr;
    bool quiet = false;  // a stopping rank with nothing pending: no stall warning while it waits
    int world() const override { return e->world_; }
    void allreduce_sum_i32(int32_t* v, int n) override {
      hipStream_t cst = e->ctrl_stream_.stream();
      TORCH_CHECK(n <= e->ctrl_dev_.numel(), "engine: control vector too long");
      hip_check(hipStreamWaitEvent(cst, e->data_ev_, 0), "hipStreamWaitEvent");
      hip_check(hipMemcpyAsync(e->ctrl_dev_.data_ptr(), v, (size_t)n * 4, hipMemcpyHostToDevice, cst), "H2D");
      std::string err;
      if (rccl_all_reduce_raw(e->ctrl_dev_.data_ptr(), (size_t)n, ncclInt32, ncclSum, e->ctrl_comm_, cst, &err) != 0)
        throw std::runtime_error("negotiation allreduce: " + err);
      hip_check(hipMemcpyAsync(v, e->ctrl_dev_.data_ptr(), (size_t)n * 4, hipMemcpyDeviceToHost, cst), "D2H");
      hip_check(hipEventRecord(e->ctrl_ev_, cst), "hipEventRecord");
      e->wait_ctrl(e->ctrl_ev_, quiet);
    }
    void allgather_i32(const int32_t* mine, int K, int32_t* out) override {
      hipStream_t cst = e->ctrl_stream_.stream();
      int32_t* ad = e->ann_dev_.data_ptr<int32_t>();
      const int64_t at = (int64_t)e->world_ * K;  // this rank's send block lives past the gather area
      hip_check(hipMemcpyAsync(ad + at, mine, (size_t)K * 4, hipMemcpyHostToDevice, cst), "H2D announce");
      std::string err;
      if (rccl_all_gather_raw(ad + at, ad, (size_t)K, ncclInt32, e->ctrl_comm_, cst, &err) != 0)
        throw std::runtime_error("announce all-gather: " + err);
      hip_check(hipMemcpyAsync(out, ad, (size_t)at * 4, hipMemcpyDeviceToHost, cst), "D2H announce");
      hip_check(hipEventRecord(e->ctrl_ev_, cst), "hipEventRecord");
      e->wait_ctrl(e->ctrl_ev_);
    }
  };

  void announce_round() {
    std::vector<uint32_t> fresh;
    try {
      fresh = agree_.announce_round(ctrl_);
    } catch (const ConsistentControlError& e) {
      throw ConsistentError(e.what());
    }
    std::lock_guard<std::mutex> lk(mu_);
    ++announces_;
    for (uint32_t h : fresh) {
      const int s = (int)slots_.size();
      Slot sl;
      sl.hash = h;
      slots_.push_back(std::move(sl));
      auto it = unassigned_.find(h);
      if (it != unassigned_.end()) {
        for (auto& item : it->second) slot_for_local(s, item).pending.push_back(std::move(item.req));
        unassigned_.erase(it);
      }
    }
  }

  void launch_copies(const std::vector<std::tuple<const char*, char*, int64_t>>& pieces) {
    hipStream_t st = stream_.stream();
    for (size_t i = 0; i < pieces.size(); i += kCopyMax) {
      CopyBatch b{};
      const int n = (int)std::min<size_t>(kCopyMax, pieces.size() - i);
      int64_t most = 0;
      for (int k = 0; k < n; ++k) {
        b.src[k] = std::get<0>(pieces[i + k]);
        b.dst[k] = std::get<1>(pieces[i + k]);
        b.bytes[k] = std::get<2>(pieces[i + k]);
        most = std::max(most, b.bytes[k]);
      }
      const int gx = (int)std::min<int64_t>(256, std::max<int64_t>(1, (most + 256 * 16 * 4 - 1) / (256 * 16 * 4)));
      hipLaunchKernelGGL(engine_batched_copy_kernel, dim3(gx, n), dim3(256), 0, st, b);
      hip_check(hipGetLastError(), "pack/unpack launch");
    }
  }

  void run_group(const std::vector<int>& group) {
    hipStream_t st = stream_.stream();
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
        // grown, never shrunk. Allocated with the data stream current, so the old block (whose last
        // use is on this stream) is freed stream-ordered; recordStream makes that explicit
        if (fusion_.defined()) c10::hip::HIPCachingAllocator::recordStream(fusion_.storage().data_ptr(), stream_);
        fusion_ = at::empty({std::max<int64_t>(nbytes, threshold_)},
                            at::TensorOptions().dtype(at::kByte).device(at::kCUDA, device_));
      }
      char* base = (char*)fusion_.data_ptr();
      std::vector<std::tuple<const char*, char*, int64_t>> in, out;
      int64_t off = 0;
      for (auto& r : reqs) {
        const int64_t nb = r.t.numel() * es;
        in.emplace_back((const char*)r.t.data_ptr(), base + off, nb);
        out.emplace_back((const char*)(base + off), (char*)r.t.data_ptr(), nb);
        off += nb;
      }
      launch_copies(in);  // MEMCPY_IN_FUSION_BUFFER: one launch
      total = nbytes / es;
      if (rccl_all_reduce_raw(base, (size_t)total, dt, op, comm_, st, &err) != 0)
        throw std::runtime_error("fused allreduce: " + err);
      launch_copies(out);  // MEMCPY_OUT_FUSION_BUFFER: one launch
    }
    hip_check(hipEventRecord(data_ev_, st), "hipEventRecord");
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
      event_put(r.ready);  // the data stream's wait above captured it
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
                     sl.known ? sl.name.c_str() : "(not submitted on this rank)", have, world_, age);
        std::lock_guard<std::mutex> lk(mu_);
        ++stalls_warned_;
      }
      if (abort_s_ > 0 && age > abort_s_) {
        std::fprintf(stderr, "[mihvd engine] stall on '%s' exceeded %.1f s: aborting (exit 134)\n",
                     sl.known ? sl.name.c_str() : "(not submitted on this rank)", abort_s_);
        std::fflush(stderr);
        std::_Exit(134);
      }
    }
    for (size_t s = 0; s < slots_.size(); ++s)
      if (!is_partial[s]) slots_[s].partial = slots_[s].warned = false;
  }

  void* comm_;
  void* ctrl_comm_;
  const int world_, device_;
  const int64_t threshold_;
  const double cycle_, warn_s_, abort_s_;
  const int cap_;
  c10::hip::HIPStream stream_, ctrl_stream_;
  at::Tensor ctrl_dev_, ctrl_host_, ann_dev_, ann_host_, fusion_;
  hipEvent_t ctrl_ev_ = nullptr;
  hipEvent_t data_ev_ = nullptr;  // the data stream's last collective (the control stream waits for it)
  // engine-thread state: the agreed slot table (hashes, announce queue) and each slot's payload
  SlotAgreement agree_;
  RcclCtrl ctrl_;
  std::vector<Slot> slots_;
  std::unordered_map<uint32_t, std::deque<Item>> unassigned_;
  // shared state (mu_)
  std::mutex mu_;
  std::condition_variable cv_done_, cv_work_;
  std::deque<Item> queue_;
  std::unordered_map<uint32_t, std::string> local_sig_;
  std::map<int64_t, std::shared_ptr<Handle>> handles_;
  int64_t next_id_ = 1, enqueued_ = 0;
  bool stopping_ = false;
  std::string fatal_;
  int64_t cycles_ = 0, collectives_ = 0, tensors_ = 0, fused_bytes_ = 0, stalls_warned_ = 0, wakeups_ = 0,
          idle_waits_ = 0, announces_ = 0;
  // event pool
  std::mutex pool_mu_;
  std::vector<hipEvent_t> pool_;
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

void engine_start(int64_t comm, int64_t ctrl_comm, int64_t fusion_bytes, double cycle_s, double warn_s,
                  double abort_s, int64_t max_slots) {
  TORCH_CHECK(fusion_bytes > 0 && cycle_s > 0 && max_slots > 0, "engine_start: bad arguments");
  std::lock_guard<std::mutex> lk(g_emu);
  TORCH_CHECK(g_engine == nullptr, "engine_start: an engine is already running");
  g_engine = std::make_unique<Engine>(comm, ctrl_comm, fusion_bytes, cycle_s, warn_s, abort_s, max_slots);
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

// CPU-testable planning step: `ctrl` is a summed control vector (int32 [2 + 2 S]), `hash` the slot
// hashes (int64, low 32 bits), `bytes` / `key` per slot. Returns the grouped ready slots (-1 ends a
// group), -2 followed by the partial slots; throws on a signature mismatch.
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

// CPU-testable slot agreement: `gathered` = the all-gathered announce blocks (int32 [world x K]),
// `assigned` = hashes that already have slots. Returns the hashes appended as new slots, in order.
std::vector<int64_t> engine_assign(const at::Tensor& gathered, int64_t world, const at::Tensor& assigned) {
  auto g = gathered.to(at::kInt).contiguous();
  TORCH_CHECK(world >= 1 && g.numel() % world == 0, "engine_assign: gathered must hold world x K entries");
  auto a = assigned.to(at::kLong).contiguous();
  std::unordered_set<uint32_t> as;
  for (int64_t i = 0; i < a.numel(); ++i) as.insert((uint32_t)a.data_ptr<int64_t>()[i]);
  const auto fresh = engine_new_slot_order(g.data_ptr<int32_t>(), (int)world, (int)(g.numel() / world), as);
  return std::vector<int64_t>(fresh.begin(), fresh.end());
}

int64_t engine_signature_hash(const std::string& sig) { return (int64_t)fnv32(sig); }

}  // namespace mihvd

TORCH_LIBRARY_FRAGMENT(mihvd, m) {
  m.def(
      "engine_start(int comm, int ctrl_comm, int fusion_bytes, float cycle_s, float warn_s, float abort_s, "
      "int max_slots) -> ()",
      &mihvd::engine_start);
  m.def("engine_allreduce_async(Tensor(a!) t, str name, int op=0) -> int", &mihvd::engine_allreduce_async);
  m.def("engine_wait(int handle) -> ()", &mihvd::engine_wait);
  m.def("engine_poll(int handle) -> bool", &mihvd::engine_poll);
  m.def("engine_stats() -> int[]", &mihvd::engine_stats);
  m.def("engine_stop() -> ()", &mihvd::engine_stop);
  m.def("engine_running() -> bool", &mihvd::engine_running);
  m.def("engine_plan(Tensor ctrl, int world, Tensor hash, Tensor bytes, Tensor key, int threshold) -> int[]",
        &mihvd::engine_plan);
  m.def("engine_assign(Tensor gathered, int world, Tensor assigned) -> int[]", &mihvd::engine_assign);
  m.def("engine_signature_hash(str sig) -> int", &mihvd::engine_signature_hash);
}
