// Direct xGMI one-shot allreduce over hipIpc-shared device buffers.
//
// the "optional xGMI direct allreduce" next to RCCL. Horovod's MPI and
// NCCL paths (reached from horovod/tensorflow_mnist.py:133 via hvd.DistributedOptimizer) always go
// through a ring; on an MI355X node every GPU has a point-to-point xGMI link to every other GPU,
// so for the latency-bound messages of this workload (the <1 MB gradient buckets of a B=100 MNIST
// step) one-shot is the better shape: every rank reads all peers' copies over its own links in
// parallel and sums them locally — one hop, no ring latency chain.
//
// Each rank owns one hipMalloc'd region, exported with hipIpcGetMemHandle and opened by every peer:
//
//     [ flags page: u32 flag[kMaxRanks] (written by peers) | u32 ctr | u32 err ] [ slot 0 ] [ slot 1 ]
//
// One call = three stream-ordered launches, all graph-capturable (the epoch lives on the device):
//   stage    copy the input into this rank's slot (ctr+1)&1
//   barrier  one wave: system release fence (+ explicit vmcnt wait, MI355X_MICROARCH.md "compiler
//            hazard"), store epoch ctr+1 into flag[rank] of every peer (system-scope atomics over
//            xGMI), poll until all peers' epochs arrived (bounded: sets err after a timeout instead
//            of hanging the GPU), then ctr += 1
//   reduce   out[i] = scale * sum_r peer_r.slot[i] in rank order (bitwise identical on every rank),
//            float4 grid-stride, all peers read concurrently over their own links. The kernel
//            boundary after the barrier is the acquire (dispatch-level system-scope invalidate).
// Double-buffered slots make one barrier per call enough: the slot written at epoch e+2 was last
// read at epoch e, and every peer finished that read before it could arrive at barrier e+1.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <torch/library.h>

#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <vector>

namespace mihvd {
namespace {

constexpr int kMaxRanks = 8;
constexpr size_t kFlagBytes = 4096;
constexpr size_t kCtrOff = 256;  // u32 epoch counter (local)
constexpr size_t kErrOff = 260;  // u32 timeout flag (local)
constexpr uint64_t kTimeoutTicks = 20ull * 100000000ull;  // 20 s of the 100 MHz wall clock

struct Peers {
  const float* data[kMaxRanks];  // each peer's slot 0
  unsigned* flags[kMaxRanks];    // each peer's flag array
};

struct Ctx {
  int device = -1, rank = 0, world = 1;
  int64_t cap = 0;  // floats per slot
  char* base = nullptr;
  Peers peers{};
  bool open = false;
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

__global__ void __launch_bounds__(256) xgmi_stage_kernel(const float* __restrict__ in, char* base, int64_t cap,
                                                         int64_t n) {
  const unsigned e = *(const volatile unsigned*)(base + kCtrOff) + 1u;
  float* dst = (float*)(base + kFlagBytes) + (int64_t)(e & 1u) * cap;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    ((float4*)dst)[i] = ((const float4*)in)[i];
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = in[i];
}

__global__ void __launch_bounds__(64) xgmi_barrier_kernel(Peers p, char* base, int world, int rank) {
  unsigned* ctr = (unsigned*)(base + kCtrOff);
  const unsigned e = *(volatile unsigned*)ctr + 1u;
  const int t = threadIdx.x;
  __atomic_thread_fence(__ATOMIC_RELEASE);  // staged slot visible system-wide before the signal
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (t < world) {
    __hip_atomic_store(p.flags[t] + rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned* mine = (const unsigned*)base + t;
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > kTimeoutTicks) {
        atomicOr((unsigned*)(base + kErrOff), 1u << t);
        break;
      }
    }
  }
  __syncthreads();
  if (t == 0) *(volatile unsigned*)ctr = e;
}

template <int W>
__global__ void __launch_bounds__(256) xgmi_reduce_kernel(Peers p, const char* base, int64_t cap, float* __restrict__ out,
                                                          int64_t n, float scale) {
  const unsigned e = *(const volatile unsigned*)(base + kCtrOff);
  const int64_t off = (int64_t)(e & 1u) * cap;
  const int64_t n4 = n >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v[W];
#pragma unroll
    for (int r = 0; r < W; ++r) v[r] = ((const float4*)(p.data[r] + off))[i];  // all loads in flight
    float4 a = v[0];
#pragma unroll
    for (int r = 1; r < W; ++r) {
      a.x += v[r].x; a.y += v[r].y; a.z += v[r].z; a.w += v[r].w;
    }
    a.x *= scale; a.y *= scale; a.z *= scale; a.w *= scale;
    ((float4*)out)[i] = a;
  }
  for (int64_t i = (n4 << 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float a = p.data[0][off + i];
#pragma unroll
    for (int r = 1; r < W; ++r) a += p.data[r][off + i];
    out[i] = a * scale;
  }
}

int grid_for_n(int64_t n) {
  int64_t g = (n / 4 + 255) / 256;  // one float4 per thread per pass
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;  // 8 blocks per CU over 256 CUs, grid-stride beyond
  return (int)g;
}

}  // namespace

int64_t xgmi_create(int64_t device, int64_t cap_floats, int64_t rank, int64_t world) {
  TORCH_CHECK(world >= 1 && world <= kMaxRanks, "xgmi: world size must be 1..", kMaxRanks);
  TORCH_CHECK(rank >= 0 && rank < world, "xgmi: bad rank");
  TORCH_CHECK(cap_floats > 0, "xgmi: capacity must be positive");
  auto* c = new Ctx();
  c->device = (int)device;
  c->rank = (int)rank;
  c->world = (int)world;
  c->cap = (cap_floats + 63) / 64 * 64;
  XGMI_HIP(hipSetDevice(c->device));
  const size_t bytes = kFlagBytes + 2 * (size_t)c->cap * sizeof(float);
  XGMI_HIP(hipMalloc((void**)&c->base, bytes));
  XGMI_HIP(hipMemset(c->base, 0, bytes));
  XGMI_HIP(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(g_mu);
  g_ctx.push_back(c);
  return (int64_t)g_ctx.size() - 1;
}

at::Tensor xgmi_handle(int64_t id) {
  Ctx* c = get(id);
  hipIpcMemHandle_t h;
  XGMI_HIP(hipSetDevice(c->device));
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
  XGMI_HIP(hipSetDevice(c->device));
  for (int r = 0; r < c->world; ++r) {
    char* ptr = nullptr;
    if (r == c->rank) {
      ptr = c->base;
    } else {
      hipIpcMemHandle_t h;
      std::memcpy(&h, hc.data_ptr<uint8_t>() + r * sizeof(h), sizeof(h));
      XGMI_HIP(hipIpcOpenMemHandle((void**)&ptr, h, hipIpcMemLazyEnablePeerAccess));
      c->opened.push_back(ptr);
    }
    c->peers.flags[r] = (unsigned*)ptr;
    c->peers.data[r] = (const float*)(ptr + kFlagBytes);
  }
  c->open = true;
}

void xgmi_allreduce_(int64_t id, const at::Tensor& t, double scale) {
  Ctx* c = get(id);
  TORCH_CHECK(c->open, "xgmi_allreduce_: call xgmi_open first");
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous(), "xgmi_allreduce_: contiguous fp32 GPU tensor");
  TORCH_CHECK(t.get_device() == c->device, "xgmi_allreduce_: tensor on device ", t.get_device(), ", context on ",
              c->device);
  TORCH_CHECK(t.numel() <= c->cap, "xgmi_allreduce_: ", t.numel(), " elements exceed the capacity ", c->cap);
  TORCH_CHECK(((uintptr_t)t.data_ptr() & 15) == 0, "xgmi_allreduce_: tensor must be 16-byte aligned");
  const int64_t n = t.numel();
  if (n == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  float* x = t.data_ptr<float>();
  const int g = grid_for_n(n);
  xgmi_stage_kernel<<<g, 256, 0, stream>>>(x, c->base, c->cap, n);
  xgmi_barrier_kernel<<<1, 64, 0, stream>>>(c->peers, c->base, c->world, c->rank);
  switch (c->world) {
#define XGMI_CASE(W) \
  case W: xgmi_reduce_kernel<W><<<g, 256, 0, stream>>>(c->peers, c->base, c->cap, x, n, (float)scale); break;
    XGMI_CASE(1) XGMI_CASE(2) XGMI_CASE(3) XGMI_CASE(4) XGMI_CASE(5) XGMI_CASE(6) XGMI_CASE(7) XGMI_CASE(8)
#undef XGMI_CASE
  }
  XGMI_HIP(hipGetLastError());
}

int64_t xgmi_error(int64_t id) {
  Ctx* c = get(id);
  unsigned err = 0;
  XGMI_HIP(hipSetDevice(c->device));
  XGMI_HIP(hipDeviceSynchronize());
  XGMI_HIP(hipMemcpy(&err, c->base + kErrOff, sizeof(err), hipMemcpyDeviceToHost));
  return (int64_t)err;
}

void xgmi_destroy(int64_t id) {
  Ctx* c = get(id);
  XGMI_HIP(hipSetDevice(c->device));
  XGMI_HIP(hipDeviceSynchronize());
  for (void* p : c->opened) (void)hipIpcCloseMemHandle(p);
  (void)hipFree(c->base);
  std::lock_guard<std::mutex> lk(g_mu);
  g_ctx[id] = nullptr;
  delete c;
}

}  // namespace mihvd

TORCH_LIBRARY_FRAGMENT(mihvd, m) {
  m.def("xgmi_create(int device, int cap_floats, int rank, int world) -> int", &mihvd::xgmi_create);
  m.def("xgmi_handle(int ctx) -> Tensor", &mihvd::xgmi_handle);
  m.def("xgmi_open(int ctx, Tensor handles) -> ()", &mihvd::xgmi_open);
  m.def("xgmi_allreduce_(int ctx, Tensor(a!) t, float scale) -> ()", &mihvd::xgmi_allreduce_);
  m.def("xgmi_error(int ctx) -> int", &mihvd::xgmi_error);
  m.def("xgmi_destroy(int ctx) -> ()", &mihvd::xgmi_destroy);
}
