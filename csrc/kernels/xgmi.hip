// Direct xGMI collectives over hipIpc-shared device memory (the node-local data plane next to RCCL).
//
// the "optional xGMI direct allreduce / gather" beside RCCL. Horovod's
// MPI and NCCL paths (reached from horovod/tensorflow_mnist.py:133 via hvd.DistributedOptimizer)
// always go through a ring; on an MI355X node every GPU has a point-to-point xGMI link to every
// other GPU, so for the latency-bound messages of this workload (sub-MB factor gathers and gradient
// buckets of a B=100 MNIST step) the one-shot shape is shorter: every rank reads all peers' copies
// over its own links at once and combines them locally — one hop, no ring latency chain.
//
// A context is one hipMalloc'd region per rank, exported with hipIpcGetMemHandle and opened by every
// peer, with the same layout on every rank:
//
//   [0, 4 KB) control  flags  u32[kPhases][kMaxRanks]  flags[ph][src] = last epoch rank src entered
//                                                       phase ph with (stored by src over xGMI)
//                      epoch  u32[kPhases]             last completed epoch of each phase (local)
//                      ticket u32[kPhases]             blocks finished in the running launch (local)
//                      err    u32                      bit r: timed out waiting for rank r; bit 31:
//                                                       this context is poisoned
//   [4 KB, ...)  data  tensors handed to torch (xgmi_view) at fixed offsets, so a peer's copy of a
//                      buffer sits at the same offset of that peer's region
//
// Every collective is ONE launch that (1) enters the phase: each block stores epoch e into
// flags[ph][rank] of every peer (system-scope stores; a block that is resident signals, so no
// residency assumption is needed), then polls its own flags[ph][*] until every peer reached e
// (bounded: a timeout sets err instead of hanging the GPU); (2) moves the data with system-scope
// loads (sc0 sc1, MI355X buffer loads with aux = 17: they miss in this GPU's L1/L2 for peer memory,
// so no line cached from an earlier epoch can be returned); (3) leaves the phase: the last block to
// finish (device-scope ticket) advances epoch[ph]. Once err is set every later launch skips the
// wait and writes NaN into its outputs (fail loudly; the host reads err at its sync points).
//
// What "entered phase ph at epoch e" promises the peers: the data this rank publishes for ph was
// written by kernels that completed before this launch began (the kernel boundary writes this
// GPU's L2s back, so a peer's xGMI read sees it), and every earlier phase launch of this context
// on this rank's stream completed, i.e. this rank finished reading the peers' data of all earlier
// phases. Callers order their buffer rewrites after a later phase (docs/ARCHITECTURE.md, "xGMI").
//
// All launches are graph-capturable: epochs live on the device.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace mihvd {
namespace {

constexpr int kMaxRanks = 8;
constexpr int kPhases = 64;
constexpr size_t kCtlBytes = 4096;
constexpr size_t kFlagsOff = 0;                                        // u32[kPhases][kMaxRanks]
constexpr size_t kEpochOff = kFlagsOff + kPhases * kMaxRanks * 4;      // 2048
constexpr size_t kTicketOff = kEpochOff + kPhases * 4;                  // 2304
constexpr size_t kErrOff = kTicketOff + kPhases * 4;                    // 2560
constexpr unsigned kPoison = 0x80000000u;
constexpr int kAuxSys = 17;  // sc0 | sc1: system-scope load (misses in L1 and in L2 for peer memory)

struct PeerTab {
  char* base[kMaxRanks];  // every rank's region (this rank's own one at [rank])
};

struct Ctx {
  int device = -1, rank = 0, world = 1;
  size_t data_bytes = 0;
  char* base = nullptr;
  PeerTab peers{};
  bool open = false;
  uint64_t timeout_ticks = 0;
  std::vector<void*> opened;
};

std::mutex g_mu;
std::vector<Ctx*> g_ctx;

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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned* ctl_u32(char* base, size_t off) { return (unsigned*)(base + off); }

// Enter phase `ph`: signal every peer, wait for every peer. Returns the epoch and whether the data
// of this launch can be trusted (false: a peer timed out now or earlier -> poison the outputs).
__device__ __forceinline__ unsigned phase_enter(const PeerTab& pt, int ph, int rank, int world, uint64_t tmo,
                                                bool& ok) {
  __shared__ unsigned s_e, s_err;
  char* mine = pt.base[rank];
  const int t = threadIdx.x;
  if (t == 0) {
    const unsigned e = __hip_atomic_load(ctl_u32(mine, kEpochOff) + ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_e = e;
    s_err = __hip_atomic_load(ctl_u32(mine, kErrOff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (int p = 0; p < world; ++p)
      if (p != rank)
        __hip_atomic_store(ctl_u32(pt.base[p], kFlagsOff) + ph * kMaxRanks + rank, e, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const unsigned e = s_e;
  int good = s_err == 0u;
  if (good && t < world && t != rank) {
    const unsigned* f = ctl_u32(mine, kFlagsOff) + ph * kMaxRanks + t;
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > tmo) {
        __hip_atomic_fetch_or(ctl_u32(mine, kErrOff), (1u << t) | kPoison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        good = 0;
        break;
      }
    }
  }
  ok = __syncthreads_and(good) != 0;
  return e;
}

// Leave phase `ph`: the last block of the launch publishes the epoch for the next launch.
__device__ __forceinline__ void phase_exit(const PeerTab& pt, int ph, int rank, unsigned e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    char* mine = pt.base[rank];
    const unsigned tk =
        __hip_atomic_fetch_add(ctl_u32(mine, kTicketOff) + ph, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == gridDim.x - 1) {
      __hip_atomic_store(ctl_u32(mine, kTicketOff) + ph, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl_u32(mine, kEpochOff) + ph, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t peer_rsrc(const char* p, uint32_t bytes) {
  // descriptor inputs are kernel arguments: wave-uniform, no waterfall loop
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// Gather rows of every peer's copy of a [world*R][row_bytes] buffer (row stride `stride` bytes,
// columns [col_off, col_off + col_bytes)) into this rank's copy: rank p's rows are [p*R, (p+1)*R),
// rows >= total_rows are skipped. All 16-byte units. W = world size (loads of all peers in flight).
template <int W>
__global__ void __launch_bounds__(256) xgmi_gather_kernel(PeerTab pt, int ph, int rank, uint64_t tmo, int64_t off,
                                                          int64_t stride, int R, int total_rows, int64_t col_off,
                                                          int64_t col_bytes) {
  bool ok;
  const unsigned e = phase_enter(pt, ph, rank, W, tmo, ok);
  const int64_t cu = col_bytes >> 4;
  const int64_t U = (int64_t)R * cu;
  const uint32_t span = (uint32_t)((int64_t)total_rows * stride);  // bytes of the buffer from `off`
  char* mine = pt.base[rank] + off;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U; i += nthreads) {
    const int64_t r = i / cu, c = i - r * cu;
    // every rank's unit is loaded (this rank's own rows too: a branch around a load makes hipcc
    // wait for each load before issuing the next); rows past total_rows read 0 (range check)
    u32x4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const uint32_t o = (uint32_t)(((int64_t)p * R + r) * stride + col_off + c * 16);
      v[p] = __builtin_amdgcn_raw_buffer_load_b128(peer_rsrc(pt.base[p] + off, span), o, 0, kAuxSys);
    }
#pragma unroll
    for (int p = 0; p < W; ++p) {
      if (p == rank) continue;
      const int64_t row = (int64_t)p * R + r;
      if (row >= total_rows) continue;
      u32x4 x = v[p];
      if (!ok) x = u32x4{0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u};  // bf16 / f32 NaN pattern
      *(u32x4*)(mine + row * stride + col_off + c * 16) = x;
    }
  }
  phase_exit(pt, ph, rank, e);
}

// Stage `in` into this rank's slot of parity (epoch+1)&1 at [slot_off + parity*slot_bytes).
__global__ void __launch_bounds__(256) xgmi_stage_kernel(const float* __restrict__ in, char* base, int ph,
                                                         int64_t slot_off, int64_t slot_bytes, int64_t n) {
  const unsigned e = __hip_atomic_load(ctl_u32(base, kEpochOff) + ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  float* dst = (float*)(base + slot_off + (int64_t)(e & 1u) * slot_bytes);
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    ((float4*)dst)[i] = ((const float4*)in)[i];
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = in[i];
}

// out[i] = scale * sum_r peer_r[src_off + parity*slot_bytes + i] in rank order (bitwise identical
// on every rank). slot_bytes = 0: a fixed buffer of the region; > 0: the staged double-buffered slot.
template <int W>
__global__ void __launch_bounds__(256) xgmi_reduce_kernel(PeerTab pt, int ph, int rank, uint64_t tmo, int64_t src_off,
                                                          int64_t slot_bytes, float* __restrict__ out, int64_t n,
                                                          float scale) {
  bool ok;
  const unsigned e = phase_enter(pt, ph, rank, W, tmo, ok);
  const int64_t off = src_off + (int64_t)(e & 1u) * slot_bytes;
  const uint32_t span = (uint32_t)(n * 4);
  const float nan = __uint_as_float(0x7FC00000u);
  const int64_t n4 = n >> 2;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += nthreads) {
    u32x4 v[W];
#pragma unroll
    for (int p = 0; p < W; ++p)
      v[p] = __builtin_amdgcn_raw_buffer_load_b128(peer_rsrc(pt.base[p] + off, span), (uint32_t)(i * 16), 0, kAuxSys);
    float4 a = make_float4(__uint_as_float(v[0].x), __uint_as_float(v[0].y), __uint_as_float(v[0].z),
                           __uint_as_float(v[0].w));
#pragma unroll
    for (int p = 1; p < W; ++p) {
      a.x += __uint_as_float(v[p].x);
      a.y += __uint_as_float(v[p].y);
      a.z += __uint_as_float(v[p].z);
      a.w += __uint_as_float(v[p].w);
    }
    a.x *= scale; a.y *= scale; a.z *= scale; a.w *= scale;
    if (!ok) a = make_float4(nan, nan, nan, nan);
    ((float4*)out)[i] = a;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += nthreads) {
    float a = 0.f;
#pragma unroll
    for (int p = 0; p < W; ++p)
      a += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(peer_rsrc(pt.base[p] + off, span), (uint32_t)(i * 4), 0,
                                                                 kAuxSys));
    out[i] = ok ? a * scale : nan;
  }
  phase_exit(pt, ph, rank, e);
}

int blocks_for(int64_t units) {
  int64_t g = (units + 255) / 256;  // one 16-byte unit per thread per pass
  if (g < 1) g = 1;
  if (g > 512) g = 512;             // two blocks per CU, grid-stride beyond
  return (int)g;
}

void check_phase(int64_t ph) { TORCH_CHECK(ph >= 0 && ph < kPhases, "xgmi: phase must be in [0, ", kPhases, ")"); }

}  // namespace

int64_t xgmi_create(int64_t device, int64_t data_bytes, int64_t rank, int64_t world) {
  TORCH_CHECK(world >= 1 && world <= kMaxRanks, "xgmi: world size must be 1..", kMaxRanks);
  TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
  TORCH_CHECK(data_bytes > 0 && data_bytes < (int64_t(1) << 32) - (int64_t)kCtlBytes,
              "xgmi: region size must be in (0, 4 GB)");
  c10::hip::HIPGuard guard((c10::DeviceIndex)device);
  auto* c = new Ctx();
  c->device = (int)device;
  c->rank = (int)rank;
  c->world = (int)world;
  c->data_bytes = ((size_t)data_bytes + 255) / 256 * 256;
  const char* tm = std::getenv("MIHVD_XGMI_TIMEOUT_MS");
  const double ms = tm ? std::atof(tm) : 20000.0;
  c->timeout_ticks = (uint64_t)((ms > 0 ? ms : 20000.0) * 1e5);  // wall_clock64 runs at 100 MHz
  const size_t bytes = kCtlBytes + c->data_bytes;
  XGMI_HIP(hipMalloc((void**)&c->base, bytes));
  XGMI_HIP(hipMemset(c->base, 0, bytes));
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
  return at::from_blob(c->base + kCtlBytes + offset, {numel}, [](void*) {}, opts);
}

void xgmi_gather_(int64_t id, int64_t ph, int64_t offset, int64_t stride, int64_t rows_per_rank, int64_t total_rows,
                  int64_t col_off, int64_t col_bytes) {
  Ctx* c = get(id);
  TORCH_CHECK(c->open, "xgmi_gather_: call xgmi_open first");
  check_phase(ph);
  TORCH_CHECK(offset % 16 == 0 && stride % 16 == 0 && col_off % 16 == 0 && col_bytes % 16 == 0,
              "xgmi_gather_: offsets, row stride and column range must be multiples of 16 bytes");
  TORCH_CHECK(col_off >= 0 && col_bytes >= 0 && col_off + col_bytes <= stride, "xgmi_gather_: bad column range");
  TORCH_CHECK(rows_per_rank >= 0 && total_rows >= 0 && total_rows <= rows_per_rank * c->world,
              "xgmi_gather_: bad row counts");
  TORCH_CHECK(offset >= 0 && offset + total_rows * stride <= (int64_t)c->data_bytes,
              "xgmi_gather_: buffer exceeds the region");
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const int g = blocks_for(rows_per_rank * (col_bytes / 16));
  const int64_t off = (int64_t)kCtlBytes + offset;
  switch (c->world) {
#define XGMI_CASE(W)                                                                                             \
  case W:                                                                                                        \
    xgmi_gather_kernel<W><<<g, 256, 0, stream>>>(c->peers, (int)ph, c->rank, c->timeout_ticks, off, stride,      \
                                                 (int)rows_per_rank, (int)total_rows, col_off, col_bytes); \
    break;
    XGMI_CASE(1) XGMI_CASE(2) XGMI_CASE(3) XGMI_CASE(4) XGMI_CASE(5) XGMI_CASE(6) XGMI_CASE(7) XGMI_CASE(8)
#undef XGMI_CASE
  }
  XGMI_HIP(hipGetLastError());
}

static void launch_reduce(Ctx* c, int64_t ph, int64_t src_off, int64_t slot_bytes, float* out, int64_t n, double scale,
                          hipStream_t stream) {
  const int g = blocks_for((n + 3) / 4);
  switch (c->world) {
#define XGMI_CASE(W)                                                                                                 \
  case W:                                                                                                            \
    xgmi_reduce_kernel<W><<<g, 256, 0, stream>>>(c->peers, (int)ph, c->rank, c->timeout_ticks, src_off, slot_bytes, \
                                                 out, n, (float)scale);                                              \
    break;
    XGMI_CASE(1) XGMI_CASE(2) XGMI_CASE(3) XGMI_CASE(4) XGMI_CASE(5) XGMI_CASE(6) XGMI_CASE(7) XGMI_CASE(8)
#undef XGMI_CASE
  }
  XGMI_HIP(hipGetLastError());
}

// Zero-copy allreduce of a region buffer: out = scale * sum over ranks of region[offset, +n floats).
void xgmi_reduce_(int64_t id, int64_t ph, int64_t offset, at::Tensor& out, double scale) {
  Ctx* c = get(id);
  TORCH_CHECK(c->open, "xgmi_reduce_: call xgmi_open first");
  check_phase(ph);
  TORCH_CHECK(out.is_cuda() && out.dtype() == at::kFloat && out.is_contiguous() && out.get_device() == c->device,
              "xgmi_reduce_: out must be a contiguous fp32 tensor on the context's device");
  TORCH_CHECK(((uintptr_t)out.data_ptr() & 15) == 0 && offset % 16 == 0, "xgmi_reduce_: 16-byte alignment required");
  const int64_t n = out.numel();
  TORCH_CHECK(offset >= 0 && offset + n * 4 <= (int64_t)c->data_bytes, "xgmi_reduce_: buffer exceeds the region");
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  launch_reduce(c, ph, (int64_t)kCtlBytes + offset, 0, out.data_ptr<float>(), n, scale,
                c10::hip::getCurrentHIPStream().stream());
}

// Allreduce of an arbitrary fp32 tensor: stage it into the double-buffered slot pair at
// [slot_off, slot_off + 2*slot_bytes) of the region, then one reduce launch back into `t`.
void xgmi_allreduce_(int64_t id, int64_t ph, at::Tensor& t, int64_t slot_off, int64_t slot_bytes, double scale) {
  Ctx* c = get(id);
  TORCH_CHECK(c->open, "xgmi_allreduce_: call xgmi_open first");
  check_phase(ph);
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous(), "xgmi_allreduce_: contiguous fp32 GPU tensor");
  TORCH_CHECK(t.get_device() == c->device, "xgmi_allreduce_: tensor on device ", t.get_device(), ", context on ",
              c->device);
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, "xgmi_allreduce_: tensor must be 16-byte aligned");
  TORCH_CHECK(slot_off % 256 == 0 && slot_bytes % 256 == 0 && slot_off + 2 * slot_bytes <= (int64_t)c->data_bytes,
              "xgmi_allreduce_: bad slot range");
  const int64_t n = t.numel();
  TORCH_CHECK(n * 4 <= slot_bytes, "xgmi_allreduce_: ", n, " elements exceed the slot capacity ", slot_bytes / 4);
  if (n == 0) return;
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  float* x = t.data_ptr<float>();
  const int64_t off = (int64_t)kCtlBytes + slot_off;
  xgmi_stage_kernel<<<blocks_for((n + 3) / 4), 256, 0, stream>>>(x, c->base, (int)ph, off, slot_bytes, n);
  XGMI_HIP(hipGetLastError());
  launch_reduce(c, ph, off, slot_bytes, x, n, scale, stream);
}

// Error word (bit r: timed out waiting for rank r; bit 31: poisoned). Waits for the current stream.
int64_t xgmi_error(int64_t id) {
  Ctx* c = get(id);
  c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  unsigned err = 0;
  XGMI_HIP(hipMemcpyAsync(&err, c->base + kErrOff, sizeof(err), hipMemcpyDeviceToHost, stream));
  XGMI_HIP(hipStreamSynchronize(stream));
  return (int64_t)err;
}

void xgmi_destroy(int64_t id) {
  Ctx* c = get(id);
  {
    c10::hip::HIPGuard guard((c10::DeviceIndex)c->device);
    XGMI_HIP(hipDeviceSynchronize());
    for (void* p : c->opened) (void)hipIpcCloseMemHandle(p);
    (void)hipFree(c->base);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_ctx[id] = nullptr;
  delete c;
}

}  // namespace mihvd

TORCH_LIBRARY_FRAGMENT(mihvd, m) {
  m.def("xgmi_create(int device, int data_bytes, int rank, int world) -> int", &mihvd::xgmi_create);
  m.def("xgmi_handle(int ctx) -> Tensor", &mihvd::xgmi_handle);
  m.def("xgmi_open(int ctx, Tensor handles) -> ()", &mihvd::xgmi_open);
  m.def("xgmi_view(int ctx, int offset, int numel, ScalarType dtype) -> Tensor", &mihvd::xgmi_view);
  m.def("xgmi_gather_(int ctx, int phase, int offset, int stride, int rows_per_rank, int total_rows, int col_off, "
        "int col_bytes) -> ()",
        &mihvd::xgmi_gather_);
  m.def("xgmi_reduce_(int ctx, int phase, int offset, Tensor(a!) out, float scale) -> ()", &mihvd::xgmi_reduce_);
  m.def("xgmi_allreduce_(int ctx, int phase, Tensor(a!) t, int slot_off, int slot_bytes, float scale) -> ()",
        &mihvd::xgmi_allreduce_);
  m.def("xgmi_error(int ctx) -> int", &mihvd::xgmi_error);
  m.def("xgmi_destroy(int ctx) -> ()", &mihvd::xgmi_destroy);
}
