// Native RCCL communicator owned by the framework ("ncclCommInitRank,
// the side stream and async-error polling in the C++ runtime").
//
// The reference's data plane is Horovod's native core (built at horovod/Dockerfile:51-65), which
// owns its NCCL communicator and enqueues the fused allreduce of every step
// (horovod/tensorflow_mnist.py:133, hvd.DistributedOptimizer) on its own stream. Here the fused
// trainer's collectives (bucket allreduce, dW3 row reduce-scatter / all-gather, state broadcast)
// go through this communicator instead of torch.distributed's process group: one RCCL comm per
// rank, created from a unique id that rank 0 draws and the ranks exchange over the bootstrap
// store, and ops that enqueue straight onto the caller's HIP stream (the trainer's side stream, or
// a stream being captured into the step's HIP graph) with no process-group bookkeeping around them.
//
// The RCCL entry points are resolved from the librccl the process already loaded (torch links it;
// /proc/self/maps names the file), so this communicator, torch's and the health monitor's view of
// them share one library instance; rccl.h is used for the types and enum values only.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <torch/library.h>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

namespace mihvd {
namespace {

struct Rccl {
  void* lib = nullptr;
  std::string path;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclCommUserRank) user_rank = nullptr;
};

std::string loaded_rccl_path() {
  std::ifstream maps("/proc/self/maps");
  std::string line;
  while (std::getline(maps, line)) {
    const auto pos = line.find('/');
    if (pos == std::string::npos) continue;
    const std::string p = line.substr(pos);
    const auto slash = p.rfind('/');
    if (p.compare(slash + 1, 9, "librccl.s") == 0) return p;
  }
  return "";
}

Rccl& rccl() {
  static std::once_flag once;
  static Rccl r;
  std::call_once(once, [] {
    std::string p = loaded_rccl_path();
    void* h = p.empty() ? nullptr : dlopen(p.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (h == nullptr) {
      p = "librccl.so.1";
      h = dlopen(p.c_str(), RTLD_NOW | RTLD_LOCAL);
    }
    if (h == nullptr) return;
    r.lib = h;
    r.path = p;
#define MIHVD_SYM(field, name) r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, #name))
    MIHVD_SYM(get_unique_id, ncclGetUniqueId);
    MIHVD_SYM(init_rank, ncclCommInitRank);
    MIHVD_SYM(destroy, ncclCommDestroy);
    MIHVD_SYM(abort, ncclCommAbort);
    MIHVD_SYM(async_error, ncclCommGetAsyncError);
    MIHVD_SYM(error_string, ncclGetErrorString);
    MIHVD_SYM(all_reduce, ncclAllReduce);
    MIHVD_SYM(all_gather, ncclAllGather);
    MIHVD_SYM(reduce_scatter, ncclReduceScatter);
    MIHVD_SYM(broadcast, ncclBroadcast);
    MIHVD_SYM(group_start, ncclGroupStart);
    MIHVD_SYM(group_end, ncclGroupEnd);
    MIHVD_SYM(send, ncclSend);
    MIHVD_SYM(recv, ncclRecv);
    MIHVD_SYM(count, ncclCommCount);
    MIHVD_SYM(user_rank, ncclCommUserRank);
#undef MIHVD_SYM
  });
  TORCH_CHECK(r.lib != nullptr && r.init_rank != nullptr && r.all_reduce != nullptr && r.all_gather != nullptr &&
                  r.reduce_scatter != nullptr && r.broadcast != nullptr && r.get_unique_id != nullptr &&
                  r.destroy != nullptr,
              "rccl_comm: librccl is not loaded in this process or lacks the expected entry points");
  return r;
}

void check(ncclResult_t e, const char* what) {
  if (e == ncclSuccess) return;
  const Rccl& r = rccl();
  TORCH_CHECK(false, "rccl_comm: ", what, " failed: ", r.error_string ? r.error_string(e) : "error", " (", (int)e,
              ")");
}

struct Comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = -1;
};

std::mutex g_mu;
std::vector<Comm*> g_comms;

Comm* get(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(h >= 0 && h < (int64_t)g_comms.size() && g_comms[h] != nullptr, "rccl_comm: bad handle ", h);
  return g_comms[h];
}

ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    default: TORCH_CHECK(false, "rccl_comm: unsupported dtype ", t.scalar_type());
  }
}

ncclRedOp_t op_of(int64_t op) {
  switch (op) {
    case 0: return ncclSum;
    case 1: return ncclProd;
    case 2: return ncclMax;
    case 3: return ncclMin;
    case 4: return ncclAvg;
    default: TORCH_CHECK(false, "rccl_comm: reduce op must be 0 sum, 1 prod, 2 max, 3 min, 4 avg");
  }
}

void check_dev(const Comm* c, const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.get_device() == c->device && t.is_contiguous(), what,
              ": expected a contiguous tensor on the communicator's device ", c->device);
}

}  // namespace

// 128-byte ncclUniqueId drawn on this rank (rank 0 shares it with the others).
at::Tensor rccl_unique_id() {
  ncclUniqueId id;
  check(rccl().get_unique_id(&id), "ncclGetUniqueId");
  auto t = at::empty({(int64_t)sizeof(id)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &id, sizeof(id));
  return t;
}

// Collective over the `world` ranks that pass the same id. Returns a handle.
int64_t rccl_comm_init(const at::Tensor& uid, int64_t rank, int64_t world, int64_t device) {
  TORCH_CHECK(uid.device().is_cpu() && uid.dtype() == at::kByte && uid.numel() == (int64_t)sizeof(ncclUniqueId),
              "rccl_comm_init: uid must be the CPU uint8[128] from rccl_unique_id");
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world, "rccl_comm_init: bad rank / world");
  ncclUniqueId id;
  std::memcpy(&id, uid.contiguous().data_ptr(), sizeof(id));
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  auto* c = new Comm();
  c->rank = (int)rank;
  c->world = (int)world;
  c->device = (int)device;
  const ncclResult_t e = rccl().init_rank(&c->comm, (int)world, id, (int)rank);
  if (e != ncclSuccess) {
    delete c;
    check(e, "ncclCommInitRank");
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

// ncclComm_t as an integer (for the health monitor's async-error polling, HealthMonitor.attach_rccl).
int64_t rccl_comm_ptr(int64_t h) { return (int64_t)(uintptr_t)get(h)->comm; }

std::string rccl_library_path() { return rccl().path; }

// What RCCL itself reports for the communicator (ncclCommCount / ncclCommUserRank), not what the
// caller passed to ncclCommInitRank: the witness bench.py prints as config.rccl_nranks.
int64_t rccl_comm_count(int64_t h) {
  Comm* c = get(h);
  TORCH_CHECK(rccl().count != nullptr, "rccl_comm_count: librccl lacks ncclCommCount");
  int n = 0;
  check(rccl().count(c->comm, &n), "ncclCommCount");
  return n;
}

int64_t rccl_comm_user_rank(int64_t h) {
  Comm* c = get(h);
  TORCH_CHECK(rccl().user_rank != nullptr, "rccl_comm_user_rank: librccl lacks ncclCommUserRank");
  int r = -1;
  check(rccl().user_rank(c->comm, &r), "ncclCommUserRank");
  return r;
}

// ---- collectives: enqueued on the current HIP stream (capturable into a HIP graph) ----
void rccl_all_reduce_(int64_t h, at::Tensor& t, int64_t op) {
  Comm* c = get(h);
  check_dev(c, t, "rccl_all_reduce_");
  if (t.numel() == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  check(rccl().all_reduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), op_of(op), c->comm, stream),
        "ncclAllReduce");
}

// out = concatenation over ranks of `in` (out may alias in at rank offset: in-place all-gather).
void rccl_all_gather(int64_t h, at::Tensor& out, const at::Tensor& in) {
  Comm* c = get(h);
  check_dev(c, out, "rccl_all_gather: out");
  check_dev(c, in, "rccl_all_gather: in");
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && out.numel() == in.numel() * c->world,
              "rccl_all_gather: out must hold world x in elements of in's dtype");
  if (in.numel() == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  check(rccl().all_gather(in.data_ptr(), out.data_ptr(), (size_t)in.numel(), dtype_of(in), c->comm, stream),
        "ncclAllGather");
}

// Several all-gathers as one RCCL group (one launch): outs[i] = concatenation over ranks of ins[i]
// (ins[i] may be this rank's block of outs[i]: in place).
void rccl_all_gather_many(int64_t h, at::TensorList outs, at::TensorList ins) {
  Comm* c = get(h);
  TORCH_CHECK(outs.size() == ins.size(), "rccl_all_gather_many: as many outputs as inputs");
  for (size_t i = 0; i < outs.size(); ++i) {
    check_dev(c, outs[i], "rccl_all_gather_many: out");
    check_dev(c, ins[i], "rccl_all_gather_many: in");
    TORCH_CHECK(outs[i].scalar_type() == ins[i].scalar_type() && outs[i].numel() == ins[i].numel() * c->world,
                "rccl_all_gather_many: out must hold world x in elements of in's dtype");
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  Rccl& r = rccl();
  check(r.group_start(), "ncclGroupStart");
  for (size_t i = 0; i < outs.size(); ++i)
    if (ins[i].numel() > 0)
      check(r.all_gather(ins[i].data_ptr(), outs[i].data_ptr(), (size_t)ins[i].numel(), dtype_of(ins[i]), c->comm,
                         stream),
            "ncclAllGather");
  check(r.group_end(), "ncclGroupEnd");
}

// out = this rank's block of the reduction over ranks of `in` (world x out elements).
void rccl_reduce_scatter(int64_t h, at::Tensor& out, const at::Tensor& in, int64_t op) {
  Comm* c = get(h);
  check_dev(c, out, "rccl_reduce_scatter: out");
  check_dev(c, in, "rccl_reduce_scatter: in");
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && in.numel() == out.numel() * c->world,
              "rccl_reduce_scatter: in must hold world x out elements of out's dtype");
  if (out.numel() == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  check(rccl().reduce_scatter(in.data_ptr(), out.data_ptr(), (size_t)out.numel(), dtype_of(out), op_of(op), c->comm,
                              stream),
        "ncclReduceScatter");
}

void rccl_broadcast_(int64_t h, at::Tensor& t, int64_t root) {
  Comm* c = get(h);
  check_dev(c, t, "rccl_broadcast_");
  TORCH_CHECK(root >= 0 && root < c->world, "rccl_broadcast_: bad root");
  if (t.numel() == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  check(rccl().broadcast(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), (int)root, c->comm, stream),
        "ncclBroadcast");
}

// Several all-reduces as one RCCL group (one launch for a list of buckets).
void rccl_all_reduce_many_(int64_t h, at::TensorList ts, int64_t op) {
  Comm* c = get(h);
  for (const auto& t : ts) check_dev(c, t, "rccl_all_reduce_many_");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  Rccl& r = rccl();
  check(r.group_start(), "ncclGroupStart");
  for (const auto& t : ts)
    if (t.numel() > 0)
      check(r.all_reduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dtype_of(t), op_of(op), c->comm, stream),
            "ncclAllReduce");
  check(r.group_end(), "ncclGroupEnd");
}

// out[j] = peer j's in[rank]: `in` and `out` are world equal blocks (block j of `in` goes to rank j),
// one RCCL group of point-to-point sends and receives (the own block is a device copy).
void rccl_all_to_all(int64_t h, at::Tensor& out, const at::Tensor& in) {
  Comm* c = get(h);
  check_dev(c, out, "rccl_all_to_all: out");
  check_dev(c, in, "rccl_all_to_all: in");
  TORCH_CHECK(out.scalar_type() == in.scalar_type() && out.numel() == in.numel() && in.numel() % c->world == 0,
              "rccl_all_to_all: in and out must hold world equal blocks of one dtype");
  TORCH_CHECK(out.data_ptr() != in.data_ptr(), "rccl_all_to_all: out must not alias in");
  if (in.numel() == 0) return;
  Rccl& r = rccl();
  TORCH_CHECK(r.send != nullptr && r.recv != nullptr && r.group_start != nullptr && r.group_end != nullptr,
              "rccl_all_to_all: librccl lacks ncclSend / ncclRecv");
  const size_t blk = (size_t)(in.numel() / c->world), bytes = blk * in.element_size();
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const char* src = static_cast<const char*>(in.data_ptr());
  char* dst = static_cast<char*>(out.data_ptr());
  const ncclDataType_t dt = dtype_of(in);
  C10_HIP_CHECK(hipMemcpyAsync(dst + c->rank * bytes, src + c->rank * bytes, bytes, hipMemcpyDeviceToDevice, stream));
  if (c->world == 1) return;
  check(r.group_start(), "ncclGroupStart");
  for (int k = 1; k < c->world; ++k) {
    // ring-ordered pairs (send to rank + k, receive from rank - k): every link carries one block
    const int to = (c->rank + k) % c->world, from = (c->rank - k + c->world) % c->world;
    check(r.send(src + to * bytes, blk, dt, to, c->comm, stream), "ncclSend");
    check(r.recv(dst + from * bytes, blk, dt, from, c->comm, stream), "ncclRecv");
  }
  check(r.group_end(), "ncclGroupEnd");
}

// One pairwise exchange as one RCCL group: `send` to rank `peer` and `recv` from it (both on the
// current stream, so the step that follows reads `recv` in stream order). The Adasum
// vector-halving / distance-doubling exchange (mihvd/parallel/adasum.py); an empty side is skipped.
void rccl_send_recv(int64_t h, const at::Tensor& send, at::Tensor& recv, int64_t peer) {
  Comm* c = get(h);
  check_dev(c, send, "rccl_send_recv: send");
  check_dev(c, recv, "rccl_send_recv: recv");
  TORCH_CHECK(peer >= 0 && peer < c->world && peer != c->rank, "rccl_send_recv: bad peer ", peer);
  TORCH_CHECK(send.scalar_type() == recv.scalar_type(), "rccl_send_recv: one dtype");
  Rccl& r = rccl();
  TORCH_CHECK(r.send != nullptr && r.recv != nullptr, "rccl_send_recv: librccl lacks ncclSend / ncclRecv");
  if (send.numel() == 0 && recv.numel() == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const ncclDataType_t dt = dtype_of(send);
  check(r.group_start(), "ncclGroupStart");
  if (send.numel() > 0) check(r.send(send.data_ptr(), (size_t)send.numel(), dt, (int)peer, c->comm, stream), "ncclSend");
  if (recv.numel() > 0) check(r.recv(recv.data_ptr(), (size_t)recv.numel(), dt, (int)peer, c->comm, stream), "ncclRecv");
  check(r.group_end(), "ncclGroupEnd");
}

// Uneven all-to-all (hvd.alltoall with splits): rows [soff[j], soff[j] + scnt[j]) of `in` (in
// elements) go to rank j, rows from rank j land at [roff[j], roff[j] + rcnt[j]) of `out`; one group
// of point-to-point transfers in ring order, the own block a device copy.
void rccl_all_to_all_v(int64_t h, at::Tensor& out, const at::Tensor& in, at::IntArrayRef scnt, at::IntArrayRef soff,
                       at::IntArrayRef rcnt, at::IntArrayRef roff) {
  Comm* c = get(h);
  check_dev(c, out, "rccl_all_to_all_v: out");
  check_dev(c, in, "rccl_all_to_all_v: in");
  TORCH_CHECK(out.scalar_type() == in.scalar_type(), "rccl_all_to_all_v: one dtype");
  const int W = c->world;
  TORCH_CHECK((int)scnt.size() == W && (int)soff.size() == W && (int)rcnt.size() == W && (int)roff.size() == W,
              "rccl_all_to_all_v: one count and offset per rank");
  for (int j = 0; j < W; ++j)
    TORCH_CHECK(scnt[j] >= 0 && soff[j] >= 0 && soff[j] + scnt[j] <= in.numel() && rcnt[j] >= 0 && roff[j] >= 0 &&
                    roff[j] + rcnt[j] <= out.numel(),
                "rccl_all_to_all_v: block ", j, " exceeds its tensor");
  TORCH_CHECK(scnt[c->rank] == rcnt[c->rank], "rccl_all_to_all_v: the own block must keep its size");
  Rccl& r = rccl();
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const size_t es = in.element_size();
  const char* src = static_cast<const char*>(in.data_ptr());
  char* dst = static_cast<char*>(out.data_ptr());
  if (scnt[c->rank] > 0)
    C10_HIP_CHECK(hipMemcpyAsync(dst + roff[c->rank] * es, src + soff[c->rank] * es, scnt[c->rank] * es,
                                 hipMemcpyDeviceToDevice, stream));
  if (W == 1) return;
  TORCH_CHECK(r.send != nullptr && r.recv != nullptr, "rccl_all_to_all_v: librccl lacks ncclSend / ncclRecv");
  const ncclDataType_t dt = dtype_of(in);
  check(r.group_start(), "ncclGroupStart");
  for (int k = 1; k < W; ++k) {
    const int to = (c->rank + k) % W, from = (c->rank - k + W) % W;
    if (scnt[to] > 0) check(r.send(src + soff[to] * es, (size_t)scnt[to], dt, to, c->comm, stream), "ncclSend");
    if (rcnt[from] > 0) check(r.recv(dst + roff[from] * es, (size_t)rcnt[from], dt, from, c->comm, stream), "ncclRecv");
  }
  check(r.group_end(), "ncclGroupEnd");
}

// 0 healthy, else the ncclResult_t of an asynchronous failure of the communicator.
int64_t rccl_async_error(int64_t h) {
  Comm* c = get(h);
  if (rccl().async_error == nullptr) return 0;
  ncclResult_t e = ncclSuccess;
  check(rccl().async_error(c->comm, &e), "ncclCommGetAsyncError");
  return e == ncclInProgress ? 0 : (int64_t)e;
}

// ---- for the native engine (engine.cpp): raw access on the engine's own stream ----
void* rccl_comm_raw(int64_t h) { return (void*)get(h)->comm; }
int rccl_comm_world(int64_t h) { return get(h)->world; }
int rccl_comm_device(int64_t h) { return get(h)->device; }

// 0 on success; otherwise the ncclResult_t with its message in *err
int rccl_all_reduce_raw(void* buf, size_t count, int dtype, int op, void* comm, hipStream_t stream, std::string* err) {
  if (count == 0) return 0;
  Rccl& r = rccl();
  const ncclResult_t e =
      r.all_reduce(buf, buf, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, (ncclComm_t)comm, stream);
  if (e != ncclSuccess && err != nullptr) *err = r.error_string ? r.error_string(e) : "RCCL error";
  return (int)e;
}

int rccl_all_gather_raw(const void* in, void* out, size_t count, int dtype, void* comm, hipStream_t stream,
                        std::string* err) {
  if (count == 0) return 0;
  Rccl& r = rccl();
  const ncclResult_t e = r.all_gather(in, out, count, (ncclDataType_t)dtype, (ncclComm_t)comm, stream);
  if (e != ncclSuccess && err != nullptr) *err = r.error_string ? r.error_string(e) : "RCCL error";
  return (int)e;
}

// ncclCommAbort of a raw communicator (the engine's local-failure path): peers blocked in a
// collective with this rank see the communicator fail instead of waiting forever
void rccl_comm_abort_raw(void* comm) {
  Rccl& r = rccl();
  if (r.abort != nullptr && comm != nullptr) (void)r.abort((ncclComm_t)comm);
}

void rccl_comm_destroy(int64_t h, bool abort) {
  Comm* c = get(h);
  {
    c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
    if (abort && rccl().abort != nullptr) (void)rccl().abort(c->comm);
    else (void)rccl().destroy(c->comm);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms[h] = nullptr;
  delete c;
}

}  // namespace mihvd

TORCH_LIBRARY_FRAGMENT(mihvd, m) {
  m.def("rccl_unique_id() -> Tensor", &mihvd::rccl_unique_id);
  m.def("rccl_comm_init(Tensor uid, int rank, int world, int device) -> int", &mihvd::rccl_comm_init);
  m.def("rccl_comm_ptr(int comm) -> int", &mihvd::rccl_comm_ptr);
  m.def("rccl_library_path() -> str", &mihvd::rccl_library_path);
  m.def("rccl_comm_count(int comm) -> int", &mihvd::rccl_comm_count);
  m.def("rccl_comm_user_rank(int comm) -> int", &mihvd::rccl_comm_user_rank);
  m.def("rccl_all_reduce_(int comm, Tensor(a!) t, int op=0) -> ()", &mihvd::rccl_all_reduce_);
  m.def("rccl_all_gather(int comm, Tensor(a!) out, Tensor input) -> ()", &mihvd::rccl_all_gather);
  m.def("rccl_all_gather_many(int comm, Tensor(a!)[] outs, Tensor[] ins) -> ()", &mihvd::rccl_all_gather_many);
  m.def("rccl_reduce_scatter(int comm, Tensor(a!) out, Tensor input, int op=0) -> ()", &mihvd::rccl_reduce_scatter);
  m.def("rccl_broadcast_(int comm, Tensor(a!) t, int root=0) -> ()", &mihvd::rccl_broadcast_);
  m.def("rccl_all_to_all(int comm, Tensor(a!) out, Tensor input) -> ()", &mihvd::rccl_all_to_all);
  m.def("rccl_all_reduce_many_(int comm, Tensor(a!)[] ts, int op=0) -> ()", &mihvd::rccl_all_reduce_many_);
  m.def("rccl_send_recv(int comm, Tensor send, Tensor(a!) recv, int peer) -> ()", &mihvd::rccl_send_recv);
  m.def("rccl_all_to_all_v(int comm, Tensor(a!) out, Tensor input, int[] scnt, int[] soff, int[] rcnt, int[] roff) -> ()",
        &mihvd::rccl_all_to_all_v);
  m.def("rccl_async_error(int comm) -> int", &mihvd::rccl_async_error);
  m.def("rccl_comm_destroy(int comm, bool abort=False) -> ()", &mihvd::rccl_comm_destroy);
}
