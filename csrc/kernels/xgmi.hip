// Direct xGMI collectives over hipIpc-shared device memory (the node-local data plane next to RCCL).
//
// the "optional xGMI direct allreduce / gather" beside RCCL. Horovod's
// MPI and NCCL paths (reached from horovod/tensorflow_mnist.py:133 via hvd.DistributedOptimizer)
// always go through a ring; on an MI355X node every GPU has a point-to-point xGMI link to every
// other GPU, so for the latency-bound messages of this workload (sub-MB factor gathers and gradient
// buckets of a B=100 MNIST step) the one-shot shape is shorter: every rank reads all peers' copies
// over its own links at once and combines them locally — one hop, no ring latency chain.
//
// A context is one hipMalloc'd region per rank (layout and phase protocol: xgmi_role.h), exported
// with hipIpcGetMemHandle and opened by every peer. Collectives are prepared once as role
// descriptors (xgmi_role_gather / xgmi_role_reduce: a CollRole with the peers' base pointers,
// offsets, phase id, timeout and optionally the fused Adam operands) and then either launched on
// their own (xgmi_run) or handed to a compute op by id, whose launch runs them on its first nblk
// blocks (co-launch: conv12_fwd, head_fwd_bwd, fc1_bwd, fc1_wgrad take a `coll` argument). Both
// forms replay from a HIP graph: the epochs live on the device and the descriptors are kernel
// arguments captured by value. xgmi_gather_/xgmi_reduce_/xgmi_allreduce_ are the one-off forms.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "xgmi_role.h"

namespace mihvd {
namespace {

struct Ctx {
  int device = -1, rank = 0, world = 1;
  size_t data_bytes = 0;
  char* base = nullptr;
  PeerTab peers{};
  bool open = false;
  uint64_t timeout_ticks = 0;
  std::vector<void*> opened;
  unsigned* herr = nullptr;      // host-coherent mirror of the error word (health monitor), or null
  unsigned* herr_dev = nullptr;  // its device address
};

std::mutex g_mu;
std::vector<Ctx*> g_ctx;
std::vector<CollRole> g_roles;
std::vector<int64_t> g_role_ctx;  // context of each descriptor (-1 once the context is destroyed)

#define XGMI_HIP(x)                                                                  \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    TORCH_CHECK(e_ == hipSuccess, "xgmi: " #x " failed: ", hipGetErrorString(e_)); \
  } while (0)

Ctx* get(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(id >= 0 && id < (int64_t)g_ctx.size() && g_ctx[id], "xgmi: bad context id ", id);
  return g_ctx[id];
}

__global__ void __launch_bounds__(256) xgmi_role_kernel(CollRole c) { coll_role_run(c, (int)blockIdx.x); }

// Split form (xgmi_role.h): the phase entry/exit of one or two collectives in one block, then a
// launch whose blocks [0, a.nblk) move a's bytes and the rest b's (the fp32 plane's small-gradient
// and dense/kernel-row reductions with their Adam updates, or its row gather alone).
__global__ void __launch_bounds__(64) xgmi_enter_kernel(CollRole a, CollRole b, int two) {
  coll_role_enter_exit(a);
  if (two) coll_role_enter_exit(b);
}

__global__ void __launch_bounds__(256) xgmi_data_kernel(CollRole a, CollRole b, int two) {
  const int bid = (int)blockIdx.x;
  if (bid < a.nblk) coll_role_data(a, bid);
  else if (two) coll_role_data(b, bid - a.nblk);
}

// Stage `in` into this rank's slot of parity (epoch+1)&1 at [slot_off + parity*slot_bytes).
__global__ void __launch_bounds__(256) xgmi_stage_kernel(const float* __restrict__ in, char* base, int ph,
                                                         int64_t slot_off, int64_t slot_bytes, int64_t n) {
  const unsigned e =
      __hip_atomic_load(xg_u32(base, kXgEpochOff) + ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  float* dst = (float*)(base + slot_off + (int64_t)(e & 1u) * slot_bytes);
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    ((float4*)dst)[i] = ((const float4*)in)[i];
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = in[i];
}

int blocks_for(int64_t units) {
  int64_t g = (units + 255) / 256;  // one 16-byte unit per thread per pass
  if (g < 1) g = 1;
  if (g > 256) g = 256;             // one block per CU, grid-stride beyond (all resident at once)
  return (int)g;
}

// Block count of a split-form data launch: one 16-byte unit per thread per pass, at most 4 blocks
// per CU (grid-stride beyond).
int data_blocks(const CollRole& r) {
  const int64_t units = r.kind == COLL_GATHER ? (int64_t)r.R * (r.col_bytes / 16) : (r.n + 3) / 4;
  int64_t g = (units + 255) / 256;
  const int64_t cap = 4 * (int64_t)device_cu_count();
  return (int)std::max<int64_t>(1, std::min(g, cap));
}

void check_phase(int64_t ph) { TORCH_CHECK(ph >= 0 && ph < kXgPhases, "xgmi: phase must be in [0, ", kXgPhases, ")"); }

CollRole base_role(Ctx* c, int64_t ph) {
  TORCH_CHECK(c->open, "xgmi: call xgmi_open first");
  check_phase(ph);
  CollRole r;
  r.pt = c->peers;
  r.ph = (int)ph;
  r.rank = c->rank;
  r.world = c->world;
  r.tmo = c->timeout_ticks;
  r.herr = c->herr_dev;
  return r;
}

CollRole gather_role(Ctx* c, int64_t ph, int64_t offset, int64_t stride, int64_t rows_per_rank, int64_t total_rows,
                     int64_t col_off, int64_t col_bytes) {
  TORCH_CHECK(offset % 16 == 0 && stride % 16 == 0 && col_off % 16 == 0 && col_bytes % 16 == 0,
              "xgmi gather: offsets, row stride and column range must be multiples of 16 bytes");
  TORCH_CHECK(col_off >= 0 && col_bytes >= 0 && col_off + col_bytes <= stride, "xgmi gather: bad column range");
  TORCH_CHECK(rows_per_rank >= 0 && total_rows >= 0 && total_rows <= rows_per_rank * c->world,
              "xgmi gather: bad row counts");
  TORCH_CHECK(offset >= 0 && offset + total_rows * stride <= (int64_t)c->data_bytes,
              "xgmi gather: buffer exceeds the region");
  CollRole r = base_role(c, ph);
  r.kind = COLL_GATHER;
  r.off = kXgCtlBytes + offset;
  r.stride = stride;
  r.R = (int)rows_per_rank;
  r.total_rows = (int)total_rows;
  r.col_off = col_off;
  r.col_bytes = col_bytes;
  r.nblk = blocks_for(rows_per_rank * (col_bytes / 16));
  const char* dbg = std::getenv("MIHVD_XGMI_DEBUG_STALE");
  r.dbg_stale = (dbg && std::atoi(dbg) != 0) ? 1 : 0;
  return r;
}

CollRole reduce_role(Ctx* c, int64_t ph, int64_t offset, int64_t slot_bytes, int64_t n, float* out, double scale) {
  TORCH_CHECK(offset % 16 == 0 && offset >= 0 &&
                  offset + (slot_bytes ? 2 * slot_bytes : n * 4) <= (int64_t)c->data_bytes,
              "xgmi reduce: buffer exceeds the region");
  CollRole r = base_role(c, ph);
  r.kind = COLL_REDUCE;
  r.off = kXgCtlBytes + offset;
  r.slot_bytes = slot_bytes;
  r.n = n;
  r.out = out;
  r.scale = (float)scale;
  r.nblk = blocks_for((n + 3) / 4);
  return r;
}

void check_out(Ctx* c, const at::Tensor& out, const char* what) {
  TORCH_CHECK(out.is_cuda() && out.dtype() == at::kFloat && out.is_contiguous() && out.get_device() == c->device &&
                  ((uintptr_t)out.data_ptr() & 15) == 0,
              what, ": out must be a 16-byte aligned contiguous fp32 tensor on the context's device");
}

void launch_role(const CollRole& r, hipStream_t stream) {
  xgmi_role_kernel<<<r.nblk, 256, 0, stream>>>(r);
  XGMI_HIP(hipGetLastError());
}

int64_t register_role(int64_t ctx, const CollRole& r) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_roles.push_back(r);
  g_role_ctx.push_back(ctx);
  return (int64_t)g_roles.size() - 1;
}

}  // namespace

CollRole xgmi_role_lookup(int64_t id) {
  if (id < 0) return CollRole{};
  std::lock_guard<std::mutex> lk(g_mu);
  TORCH_CHECK(id < (int64_t)g_roles.size() && g_role_ctx[id] >= 0, "xgmi: bad collective descriptor ", id);
  return g_roles[id];
}

int64_t xgmi_create(int64_t device, int64_t data_bytes, int64_t rank, int64_t world) {
  TORCH_CHECK(world >= 1 && world <= kXgMaxRanks, "xgmi: world size must be 1..", kXgMaxRanks);
  TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
  TORCH_CHECK(data_bytes > 0 && data_bytes < (int64_t(1) << 32) - kXgCtlBytes, "xgmi: region size must be in (0, 4 GB)");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  auto* c = new Ctx();
  c->device = (int)device;
  c->rank = (int)rank;
  c->world = (int)world;
  c->data_bytes = ((size_t)data_bytes + 255) / 256 * 256;
  const char* tm = std::getenv("MIHVD_XGMI_TIMEOUT_MS");
  const double ms = tm ? std::atof(tm) : 20000.0;
  c->timeout_ticks = (uint64_t)((ms > 0 ? ms : 20000.0) * 1e5);  // wall_clock64 runs at 100 MHz
  const size_t bytes = kXgCtlBytes + c->data_bytes;
  XGMI_HIP(hipMalloc((void**)&c->base, bytes));
  XGMI_HIP(hipMemset(c->base, 0, bytes));
  // the timeout mirror lives in fine-grained host memory: a device system-scope store reaches it
  // while kernels are still running, so the health monitor's thread sees it without a sync
  void* h = nullptr;
  if (hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess && h != nullptr) {
    std::memset(h, 0, 64);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess && d != nullptr) {
      c->herr = (unsigned*)h;
      c->herr_dev = (unsigned*)d;
    } else {
      (void)hipHostFree(h);
    }
  }
  (void)hipGetLastError();
  XGMI_HIP(hipDeviceSynchronize());
  c->peers.base[c->rank] = c->base;
  std::lock_guard<std::mutex> lk(g_mu);
  g_ctx.push_back(c);
  return (int64_t)g_ctx.size() - 1;
}

at::Tensor xgmi_handle(int64_t id) {
  Ctx* c = get(id);
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  hipIpcMemHandle_t h;
  XGMI_HIP(hipIpcGetMemHandle(&h, c->base));
  auto t = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

void xgmi_open(int64_t id, const at::Tensor& handles) {
  Ctx* c = get(id);
  TORCH_CHECK(!c->open, "xgmi_open: already open");
  TORCH_CHECK(handles.device().is_cpu() && handles.dtype() == at::kByte && handles.dim() == 2 &&
                  handles.size(0) == c->world && handles.size(1) == (int64_t)sizeof(hipIpcMemHandle_t),
              "xgmi_open: handles must be a CPU uint8 [world, sizeof(hipIpcMemHandle_t)] tensor");
  auto hc = handles.contiguous();
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  for (int r = 0; r < c->world; ++r) {
    if (r == c->rank) continue;
    hipIpcMemHandle_t h;
    std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
    char* ptr = nullptr;
    XGMI_HIP(hipIpcOpenMemHandle((void**)&ptr, h, hipIpcMemLazyEnablePeerAccess));
    c->opened.push_back(ptr);
    c->peers.base[r] = ptr;
  }
  c->open = true;
}

// A tensor over [offset, offset + numel * itemsize) of this rank's data region (no ownership: the
// context outlives its views; xgmi_destroy is the caller's last use).
at::Tensor xgmi_view(int64_t id, int64_t offset, int64_t numel, at::ScalarType dtype) {
  Ctx* c = get(id);
  const int64_t item = (int64_t)c10::elementSize(dtype);
  TORCH_CHECK(offset >= 0 && offset % 256 == 0, "xgmi_view: offset must be a non-negative multiple of 256");
  TORCH_CHECK(numel >= 0 && offset + numel * item <= (int64_t)c->data_bytes, "xgmi_view: view exceeds the region (",
              offset + numel * item, " > ", c->data_bytes, " bytes)");
  auto opts = at::TensorOptions().dtype(dtype).device(at::Device(at::kCUDA, (c10::DeviceIndex)c->device));
  return at::from_blob(c->base + kXgCtlBytes + offset, {numel}, [](void*) {}, opts);
}

// ---------------------------------------------------------------- prepared collectives
// nblk > 0 overrides the role block count (co-launch hosts size it to the CUs they leave idle).
int64_t xgmi_role_gather(int64_t id, int64_t ph, int64_t offset, int64_t stride, int64_t rows_per_rank,
                         int64_t total_rows, int64_t col_off, int64_t col_bytes, int64_t nblk) {
  Ctx* c = get(id);
  CollRole r = gather_role(c, ph, offset, stride, rows_per_rank, total_rows, col_off, col_bytes);
  if (nblk > 0) r.nblk = (int)nblk;
  return register_role(id, r);
}

int64_t xgmi_role_reduce(int64_t id, int64_t ph, int64_t offset, at::Tensor& out, double scale,
                         const c10::optional<at::Tensor>& p, const c10::optional<at::Tensor>& m,
                         const c10::optional<at::Tensor>& v, const c10::optional<at::Tensor>& shadow,
                         const c10::optional<at::Tensor>& state, double lr, double b1, double b2, double eps,
                         double grad_scale, int64_t rule, int64_t nblk) {
  Ctx* c = get(id);
  check_out(c, out, "xgmi_role_reduce");
  const int64_t n = out.numel();
  CollRole r = reduce_role(c, ph, offset, 0, n, out.data_ptr<float>(), scale);
  if (p.has_value() && p->defined()) {
    TORCH_CHECK(n % 4 == 0, "xgmi_role_reduce: with Adam the length must be a multiple of 4");
    for (const c10::optional<at::Tensor>* t : {&p, &m, &v})
      TORCH_CHECK(t->has_value() && (*t)->defined() && (*t)->is_cuda() && (*t)->dtype() == at::kFloat &&
                      (*t)->is_contiguous() && (*t)->numel() == n && ((uintptr_t)(*t)->data_ptr() & 15) == 0,
                  "xgmi_role_reduce: p, m, v must be aligned contiguous fp32 like out");
    TORCH_CHECK(shadow.has_value() && shadow->defined() && shadow->dtype() == at::kBFloat16 &&
                    shadow->is_contiguous() && shadow->numel() == n,
                "xgmi_role_reduce: shadow must be bf16 like p");
    TORCH_CHECK(state.has_value() && state->defined() && state->dtype() == at::kLong && state->numel() >= ST_WORDS &&
                    state->is_cuda(),
                "xgmi_role_reduce: state must be the int64 device step state");
    r.adam = 1;
    r.aa = AdamArgs{p->data_ptr<float>(), m->data_ptr<float>(), v->data_ptr<float>(), (u16*)shadow->data_ptr(),
                    state->data_ptr<int64_t>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale,
                    (int)rule};
  }
  if (nblk > 0) r.nblk = (int)nblk;
  return register_role(id, r);
}

// Reduce of n floats at region byte `offset` (sum over ranks, rank order, times scale) into `out`
// (optional) with the Adam update of fp32 parameters p (m, v; no bf16 copy) from the sum; `bump`:
// block 0 also advances the forward step counter. The fp32 plane's prepared reductions.
int64_t xgmi_role_reduce_f32(int64_t id, int64_t ph, int64_t offset, int64_t n, const c10::optional<at::Tensor>& out,
                             double scale, at::Tensor& p, at::Tensor& m, at::Tensor& v, const at::Tensor& state,
                             double lr, double b1, double b2, double eps, double grad_scale, int64_t rule, bool bump,
                             int64_t nblk) {
  Ctx* c = get(id);
  TORCH_CHECK(n > 0 && n % 4 == 0, "xgmi_role_reduce_f32: n must be a positive multiple of 4");
  float* o = nullptr;
  if (out.has_value() && out->defined()) {
    check_out(c, *out, "xgmi_role_reduce_f32");
    TORCH_CHECK(out->numel() == n, "xgmi_role_reduce_f32: out must hold n floats");
    o = out->data_ptr<float>();
  }
  for (const at::Tensor* t : {&p, &m, &v})
    TORCH_CHECK(t->is_cuda() && t->dtype() == at::kFloat && t->is_contiguous() && t->numel() == n &&
                    t->get_device() == c->device && ((uintptr_t)t->data_ptr() & 15) == 0,
                "xgmi_role_reduce_f32: p, m, v must be aligned contiguous fp32 tensors of n floats");
  TORCH_CHECK(state.is_cuda() && state.dtype() == at::kLong && state.numel() >= ST_WORDS,
              "xgmi_role_reduce_f32: state must be the int64 device step state");
  CollRole r = reduce_role(c, ph, offset, 0, n, o, scale);
  r.adam = 1;
  r.bump = bump ? 1 : 0;
  r.aa = AdamArgs{p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), nullptr, state.data_ptr<int64_t>(),
                  (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale, (int)rule};
  if (nblk > 0) r.nblk = (int)nblk;
  return register_role(id, r);
}

// One or two prepared collectives (different phases) in the split form on the current stream: a
// one-block entry launch, then one data launch. role_b < 0: one collective. `in_step` keeps the
// debug stale-read injection (a launch of the training step; see xgmi_run). `enter` = false: the
// data launch alone (a world of one, which has no peer to wait for).
void xgmi_run_split(int64_t role_a, int64_t role_b, bool in_step, bool enter) {
  CollRole a = xgmi_role_lookup(role_a);
  const bool two = role_b >= 0;
  CollRole b = two ? xgmi_role_lookup(role_b) : a;
  TORCH_CHECK(a.kind != COLL_NONE && b.kind != COLL_NONE && a.nblk > 0 && b.nblk > 0,
              "xgmi_run_split: empty descriptor");
  TORCH_CHECK(!two || a.ph != b.ph, "xgmi_run_split: the two collectives need different phases");
  if (!in_step) a.dbg_stale = b.dbg_stale = 0;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  if (enter) {
    xgmi_enter_kernel<<<1, 64, 0, stream>>>(a, b, two ? 1 : 0);
    XGMI_HIP(hipGetLastError());
  }
  // The data blocks never wait (the entry launch did), so they need not all be resident: up to
  // four per CU (16 waves) keep enough loads in flight for a memory-bound sum + Adam, where the
  // co-launch cap of one block per CU left 4 waves per CU each walking its units one round trip
  // at a time.
  a.nblk = data_blocks(a);
  if (two) b.nblk = data_blocks(b);
  xgmi_data_kernel<<<a.nblk + (two ? b.nblk : 0), 256, 0, stream>>>(a, b, two ? 1 : 0);
  XGMI_HIP(hipGetLastError());
}

// Launch a prepared collective on its own (current stream).
// `in_step`: a launch of the training step (the fp32 plane's row gather), which keeps the debug
// stale-read injection; otherwise a standalone launch (start-up validation) that stays exact.
void xgmi_run(int64_t role, bool in_step) {
  CollRole r = xgmi_role_lookup(role);
  TORCH_CHECK(r.kind != COLL_NONE && r.nblk > 0, "xgmi_run: empty descriptor");
  // the debug stale-read injection models in-step staleness only: standalone launches (the
  // start-up validation, _validate_xgmi) stay exact, so the end-to-end check must catch it
  if (!in_step) r.dbg_stale = 0;
  launch_role(r, c10::hip::getCurrentHIPStream().stream());
}

// ---------------------------------------------------------------- one-off forms
void xgmi_gather_(int64_t id, int64_t ph, int64_t offset, int64_t stride, int64_t rows_per_rank, int64_t total_rows,
                  int64_t col_off, int64_t col_bytes) {
  Ctx* c = get(id);
  CollRole r = gather_role(c, ph, offset, stride, rows_per_rank, total_rows, col_off, col_bytes);
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  launch_role(r, c10::hip::getCurrentHIPStream().stream());
}

// Zero-copy allreduce of a region buffer: out = scale * sum over ranks of region[offset, +n floats).
void xgmi_reduce_(int64_t id, int64_t ph, int64_t offset, at::Tensor& out, double scale) {
  Ctx* c = get(id);
  check_out(c, out, "xgmi_reduce_");
  CollRole r = reduce_role(c, ph, offset, 0, out.numel(), out.data_ptr<float>(), scale);
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  launch_role(r, c10::hip::getCurrentHIPStream().stream());
}

// Allreduce of an arbitrary fp32 tensor: stage it into the double-buffered slot pair at
// [slot_off, slot_off + 2*slot_bytes) of the region, then one reduce launch back into `t`.
void xgmi_allreduce_(int64_t id, int64_t ph, at::Tensor& t, int64_t slot_off, int64_t slot_bytes, double scale) {
  Ctx* c = get(id);
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous(), "xgmi_allreduce_: contiguous fp32 GPU tensor");
  TORCH_CHECK(t.get_device() == c->device, "xgmi_allreduce_: tensor on device ", t.get_device(), ", context on ",
              c->device);
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, "xgmi_allreduce_: tensor must be 16-byte aligned");
  TORCH_CHECK(slot_off % 256 == 0 && slot_bytes % 256 == 0 && slot_off + 2 * slot_bytes <= (int64_t)c->data_bytes,
              "xgmi_allreduce_: bad slot range");
  const int64_t n = t.numel();
  TORCH_CHECK(n * 4 <= slot_bytes, "xgmi_allreduce_: ", n, " elements exceed the slot capacity ", slot_bytes / 4);
  if (n == 0) return;
  CollRole r = reduce_role(c, ph, slot_off, slot_bytes, n, t.data_ptr<float>(), scale);
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  xgmi_stage_kernel<<<blocks_for((n + 3) / 4), 256, 0, stream>>>(t.data_ptr<float>(), c->base, (int)ph,
                                                                 kXgCtlBytes + slot_off, slot_bytes, n);
  XGMI_HIP(hipGetLastError());
  launch_role(r, stream);
}

// Error word (bit r: timed out waiting for rank r; bit 31: poisoned). Waits for the current stream.
int64_t xgmi_error(int64_t id) {
  Ctx* c = get(id);
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  unsigned err = 0;
  XGMI_HIP(hipMemcpyAsync(&err, c->base + kXgErrOff, sizeof(err), hipMemcpyDeviceToHost, stream));
  XGMI_HIP(hipStreamSynchronize(stream));
  return (int64_t)err;
}

// Host address of the error word's host-coherent mirror (0: none), for HealthMonitor.watch_word.
int64_t xgmi_error_word(int64_t id) { return (int64_t)(uintptr_t)get(id)->herr; }

void xgmi_destroy(int64_t id) {
  Ctx* c = get(id);
  {
    c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
    XGMI_HIP(hipDeviceSynchronize());
    for (void* p : c->opened) (void)hipIpcCloseMemHandle(p);
    (void)hipFree(c->base);
    if (c->herr != nullptr) (void)hipHostFree(c->herr);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = 0; i < g_role_ctx.size(); ++i)
    if (g_role_ctx[i] == id) g_role_ctx[i] = -1;
  g_ctx[id] = nullptr;
  delete c;
}

}  // namespace mihvd

TORCH_LIBRARY_FRAGMENT(mihvd, m) {
  m.def("xgmi_create(int device, int data_bytes, int rank, int world) -> int", &mihvd::xgmi_create);
  m.def("xgmi_handle(int ctx) -> Tensor", &mihvd::xgmi_handle);
  m.def("xgmi_open(int ctx, Tensor handles) -> ()", &mihvd::xgmi_open);
  m.def("xgmi_view(int ctx, int offset, int numel, ScalarType dtype) -> Tensor", &mihvd::xgmi_view);
  m.def("xgmi_role_gather(int ctx, int phase, int offset, int stride, int rows_per_rank, int total_rows, int col_off, "
        "int col_bytes, int nblk=0) -> int",
        &mihvd::xgmi_role_gather);
  m.def("xgmi_role_reduce(int ctx, int phase, int offset, Tensor(a!) out, float scale, Tensor? p=None, Tensor? m=None, "
        "Tensor? v=None, Tensor? shadow=None, Tensor? state=None, float lr=0., float b1=0., float b2=0., float eps=0., "
        "float grad_scale=1., int rule=0, int nblk=0) -> int",
        &mihvd::xgmi_role_reduce);
  m.def("xgmi_role_reduce_f32(int ctx, int phase, int offset, int n, Tensor(a!)? out, float scale, Tensor(b!) p, "
        "Tensor(c!) m, Tensor(d!) v, Tensor state, float lr, float b1, float b2, float eps, float grad_scale, int rule, "
        "bool bump, int nblk=0) -> int",
        &mihvd::xgmi_role_reduce_f32);
  m.def("xgmi_run(int role, bool in_step=False) -> ()", &mihvd::xgmi_run);
  m.def("xgmi_run_split(int role_a, int role_b=-1, bool in_step=False, bool enter=True) -> ()",
        &mihvd::xgmi_run_split);
  m.def("xgmi_gather_(int ctx, int phase, int offset, int stride, int rows_per_rank, int total_rows, int col_off, "
        "int col_bytes) -> ()",
        &mihvd::xgmi_gather_);
  m.def("xgmi_reduce_(int ctx, int phase, int offset, Tensor(a!) out, float scale) -> ()", &mihvd::xgmi_reduce_);
  m.def("xgmi_allreduce_(int ctx, int phase, Tensor(a!) t, int slot_off, int slot_bytes, float scale) -> ()",
        &mihvd::xgmi_allreduce_);
  m.def("xgmi_error(int ctx) -> int", &mihvd::xgmi_error);
  m.def("xgmi_error_word(int ctx) -> int", &mihvd::xgmi_error_word);
  m.def("xgmi_destroy(int ctx) -> ()", &mihvd::xgmi_destroy);
}
