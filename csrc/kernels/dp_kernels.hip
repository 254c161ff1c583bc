// Data-parallel support kernels: Adasum combine and mixed-precision
// loss-scale handling (N12).
//
// Adasum (reference: --use-adasum, horovod/tensorflow_mnist.py:31-32,133) combines two gradient
// vectors per tensor ("segment"):
//     adasum(a, b) = (1 - a.b / 2|a|^2) a + (1 - a.b / 2|b|^2) b
// It needs three reductions per segment followed by an axpby, so it is two launches:
//   segment_dots  — grid (chunk, segment); each block reduces its chunk of one segment in fp32 and
//                   adds the block total into fp64 accumulators (global fp64 atomics on gfx950).
//   adasum_combine — same grid; each block turns the segment's (ab, aa, bb) into the two
//                   coefficients and streams out = ca*a + cb*b (float4 when the segment allows).
// Segments are given as an int64 table [S+1 offsets | S flags]; the host wrapper covers gaps with
// extra segments flagged "plain sum" (padding between tensors of a fusion buffer is not a tensor).
//
// Loss scaling (reference mixed_float16 policy, horovod/tensorflow_mnist_gpu.py:26-28; Keras wraps
// the optimizer in a dynamic LossScaleOptimizer) keeps its whole state on the device in a float32
// pair ls = [scale, found_nonfinite] so a step needs no host round trip:
//   grad_check_   multi-tensor pass over the gradients: optional in-place unscale by 1/ls[0] and a
//                 non-finite test that raises ls[1];
//   adam_step     (optim.hip) skips the update when ls[1] != 0 and folds 1/ls[0] into its gradient scale;
//   update_scale_ one thread: back off on overflow, grow after `interval` clean steps, clear ls[1].
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include <vector>

#include "common.h"

namespace mihvd {

constexpr int kDotThreads = 256;
constexpr int kChunk = kDotThreads * 4 * 8;  // elements per block: 8 float4 per thread

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kDotThreads / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// Per-segment [lo, hi) -> this block's chunk [c0, c1).
__device__ __forceinline__ bool chunk_of(const int64_t* offs, int64_t& c0, int64_t& c1, bool skip_sum_segments) {
  const int s = blockIdx.y;
  const int64_t lo = offs[s], hi = offs[s + 1];
  if (skip_sum_segments && offs[gridDim.y + 1 + s]) return false;  // plain-sum segment: no dots needed
  c0 = lo + (int64_t)blockIdx.x * kChunk;
  c1 = c0 + kChunk < hi ? c0 + kChunk : hi;
  return c0 < hi;
}

__global__ void __launch_bounds__(kDotThreads) segment_dots_kernel(const float* __restrict__ a,
                                                                   const float* __restrict__ b,
                                                                   const int64_t* __restrict__ offs,
                                                                   double* __restrict__ out) {
  __shared__ float red[kDotThreads / 64];
  int64_t c0, c1;
  if (!chunk_of(offs, c0, c1, true)) return;
  float ab = 0.f, aa = 0.f, bb = 0.f;
  // Scalar head until 16-byte alignment, float4 body, scalar tail: all loads of the body are
  // issued before any use (8 independent float4 per operand per thread).
  int64_t head = c0;
  while (head < c1 && (reinterpret_cast<uintptr_t>(a + head) & 15)) ++head;
  // a and b at different 16-byte phases: everything goes through the scalar loops
  if (reinterpret_cast<uintptr_t>(b + head) & 15) head = c1;
  const int64_t nb4 = (c1 - head) >> 2;
  const int64_t tail = head + (nb4 << 2);
  for (int64_t i = c0 + threadIdx.x; i < head; i += kDotThreads) {
    const float x = a[i], y = b[i];
    ab = fmaf(x, y, ab); aa = fmaf(x, x, aa); bb = fmaf(y, y, bb);
  }
  const float4* a4 = reinterpret_cast<const float4*>(a + head);
  const float4* b4 = reinterpret_cast<const float4*>(b + head);
  float4 xa[8], xb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int64_t j = threadIdx.x + (int64_t)k * kDotThreads;
    const bool in = j < nb4;
    xa[k] = in ? a4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    xb[k] = in ? b4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float* x = &xa[k].x;
    const float* y = &xb[k].x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ab = fmaf(x[e], y[e], ab); aa = fmaf(x[e], x[e], aa); bb = fmaf(y[e], y[e], bb);
    }
  }
  for (int64_t i = tail + threadIdx.x; i < c1; i += kDotThreads) {
    const float x = a[i], y = b[i];
    ab = fmaf(x, y, ab); aa = fmaf(x, x, aa); bb = fmaf(y, y, bb);
  }
  ab = block_sum(ab, red);
  aa = block_sum(aa, red);
  bb = block_sum(bb, red);
  if (threadIdx.x == 0) {
    double* o = out + 3 * blockIdx.y;
    atomicAdd(o + 0, (double)ab);
    atomicAdd(o + 1, (double)aa);
    atomicAdd(o + 2, (double)bb);
  }
}

__global__ void __launch_bounds__(kDotThreads) adasum_combine_kernel(const float* __restrict__ a,
                                                                     const float* __restrict__ b,
                                                                     const int64_t* __restrict__ offs,
                                                                     const double* __restrict__ dots,
                                                                     float* __restrict__ out) {
  int64_t c0, c1;
  if (!chunk_of(offs, c0, c1, false)) return;
  const bool plain = offs[gridDim.y + 1 + blockIdx.y] != 0;
  const double ab = dots[3 * blockIdx.y], aa = dots[3 * blockIdx.y + 1], bb = dots[3 * blockIdx.y + 2];
  // |a| = 0 -> b ; |b| = 0 -> a ; both zero -> a + b (padding).
  const float ca = plain ? 1.f : bb > 0.0 ? (aa > 0.0 ? (float)(1.0 - ab / (2.0 * aa)) : 0.f) : 1.f;
  const float cb = plain ? 1.f : aa > 0.0 ? (bb > 0.0 ? (float)(1.0 - ab / (2.0 * bb)) : 0.f) : 1.f;
  const bool vec = (((c0 | c1) & 3) == 0) && ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                                                reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (vec) {
    const int64_t n4 = (c1 - c0) >> 2;
    const float4* a4 = reinterpret_cast<const float4*>(a + c0);
    const float4* b4 = reinterpret_cast<const float4*>(b + c0);
    float4* o4 = reinterpret_cast<float4*>(out + c0);
    for (int64_t j = threadIdx.x; j < n4; j += kDotThreads) {
      const float4 x = a4[j], y = b4[j];
      o4[j] = make_float4(ca * x.x + cb * y.x, ca * x.y + cb * y.y, ca * x.z + cb * y.z, ca * x.w + cb * y.w);
    }
  } else {
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kDotThreads) out[i] = ca * a[i] + cb * b[i];
  }
}

// ---------------------------------------------------------------------------------------------
// Loss scaling

constexpr int kMaxTensors = 32;
struct TensorTable {
  float* p[kMaxTensors];
  int64_t n[kMaxTensors];
};

__global__ void __launch_bounds__(256) grad_check_kernel(TensorTable tt, float* __restrict__ ls, int unscale) {
  const int t = blockIdx.y;
  float* p = tt.p[t];
  const int64_t n = tt.n[t];
  const float inv = unscale ? 1.f / ls[0] : 1.f;
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float g = p[i];
    if (unscale) {
      g *= inv;
      p[i] = g;
    }
    bad |= !isfinite(g);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) ls[1] = 1.f;
}

// state (optional, the fused fp16 step): a skipped update does not count as an optimizer step,
// like Keras' LossScaleOptimizer, so the step the head advanced is taken back
__global__ void update_scale_kernel(float* __restrict__ ls, int32_t* __restrict__ tracker, float growth, float backoff,
                                    int interval, float min_scale, int64_t* __restrict__ state) {
  if (ls[1] != 0.f) {
    ls[0] = fmaxf(ls[0] * backoff, min_scale);
    tracker[0] = 0;
    if (state != nullptr) state[ST_OPT] -= 1;
  } else if (++tracker[0] >= interval) {
    const float s = ls[0] * growth;
    if (isfinite(s)) ls[0] = s;
    tracker[0] = 0;
  }
  ls[1] = 0.f;
}

// ---------------------------------------------------------------------------------------------
// Host wrappers

static void check_f32_cuda(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous(), what, ": contiguous fp32 GPU tensor expected");
}

static int64_t max_chunks(const std::vector<int64_t>& offs) {
  int64_t m = 1;
  for (size_t s = 0; s + 1 < offs.size(); ++s) m = std::max<int64_t>(m, (offs[s + 1] - offs[s] + kChunk - 1) / kChunk);
  return m;
}

// `offs` is a host-side list (it is the static bucket layout); it is uploaded into `offs_dev` once by
// the caller (so a captured graph holds no host pointers).
void segment_dots(const at::Tensor& a, const at::Tensor& b, const at::Tensor& offs_dev, int64_t max_seg_len,
                  at::Tensor& out) {
  check_f32_cuda(a, "segment_dots(a)");
  check_f32_cuda(b, "segment_dots(b)");
  TORCH_CHECK(a.numel() == b.numel(), "segment_dots: size mismatch");
  TORCH_CHECK(offs_dev.is_cuda() && offs_dev.dtype() == at::kLong && offs_dev.dim() == 1 && offs_dev.numel() >= 3 &&
                  offs_dev.numel() % 2 == 1,
              "segment_dots: offs must be an int64 GPU vector [S+1 offsets | S plain-sum flags]");
  const int64_t S = offs_dev.numel() / 2;
  TORCH_CHECK(out.is_cuda() && out.dtype() == at::kDouble && out.numel() == 3 * S && out.is_contiguous(),
              "segment_dots: out must be fp64 [S,3]");
  TORCH_CHECK(S <= 65535, "segment_dots: too many segments");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  hipMemsetAsync(out.data_ptr(), 0, out.numel() * sizeof(double), stream);
  const dim3 grid((unsigned)std::max<int64_t>(1, (max_seg_len + kChunk - 1) / kChunk), (unsigned)S);
  segment_dots_kernel<<<grid, kDotThreads, 0, stream>>>(a.data_ptr<float>(), b.data_ptr<float>(),
                                                        offs_dev.data_ptr<int64_t>(), out.data_ptr<double>());
}

void adasum_combine(const at::Tensor& a, const at::Tensor& b, const at::Tensor& offs_dev, int64_t max_seg_len,
                    const at::Tensor& dots, at::Tensor& out) {
  check_f32_cuda(a, "adasum_combine(a)");
  check_f32_cuda(b, "adasum_combine(b)");
  check_f32_cuda(out, "adasum_combine(out)");
  TORCH_CHECK(a.numel() == b.numel() && out.numel() == a.numel(), "adasum_combine: size mismatch");
  TORCH_CHECK(offs_dev.numel() % 2 == 1 && offs_dev.numel() >= 3, "adasum_combine: offs table");
  const int64_t S = offs_dev.numel() / 2;
  TORCH_CHECK(dots.dtype() == at::kDouble && dots.numel() == 3 * S, "adasum_combine: dots must be fp64 [S,3]");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const dim3 grid((unsigned)std::max<int64_t>(1, (max_seg_len + kChunk - 1) / kChunk), (unsigned)S);
  adasum_combine_kernel<<<grid, kDotThreads, 0, stream>>>(a.data_ptr<float>(), b.data_ptr<float>(),
                                                          offs_dev.data_ptr<int64_t>(), dots.data_ptr<double>(),
                                                          out.data_ptr<float>());
}

void grad_check_(at::TensorList grads, at::Tensor& ls, bool unscale) {
  check_f32_cuda(ls, "grad_check_(ls)");
  TORCH_CHECK(ls.numel() == 2, "grad_check_: ls must be float32 [scale, found_nonfinite]");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  for (size_t base = 0; base < grads.size(); base += kMaxTensors) {
    TensorTable tt{};
    int cnt = 0;
    int64_t maxn = 1;
    for (size_t i = base; i < grads.size() && cnt < kMaxTensors; ++i, ++cnt) {
      check_f32_cuda(grads[i], "grad_check_(grad)");
      tt.p[cnt] = grads[i].data_ptr<float>();
      tt.n[cnt] = grads[i].numel();
      maxn = std::max<int64_t>(maxn, tt.n[cnt]);
    }
    const unsigned gx = (unsigned)std::min<int64_t>((maxn + 255) / 256, 1024);
    grad_check_kernel<<<dim3(gx, cnt), 256, 0, stream>>>(tt, ls.data_ptr<float>(), unscale ? 1 : 0);
  }
}

void update_scale_(at::Tensor& ls, at::Tensor& tracker, double growth, double backoff, int64_t interval,
                   double min_scale, const c10::optional<at::Tensor>& state) {
  check_f32_cuda(ls, "update_scale_(ls)");
  TORCH_CHECK(tracker.is_cuda() && tracker.dtype() == at::kInt && tracker.numel() >= 1, "update_scale_: int32 tracker");
  int64_t* sp = nullptr;
  if (state.has_value() && state->defined()) {
    TORCH_CHECK(state->is_cuda() && state->dtype() == at::kLong && state->numel() >= ST_WORDS,
                "update_scale_: state must be the int64 device step state");
    sp = state->data_ptr<int64_t>();
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  update_scale_kernel<<<1, 1, 0, stream>>>(ls.data_ptr<float>(), tracker.data_ptr<int32_t>(), (float)growth,
                                           (float)backoff, (int)interval, (float)min_scale, sp);
}

// ------------------------------------------------------------------------------------------ //
// Column-slice gather for the sharded dense/kernel optimizer's all-to-all (fused_mnist.py):
//   dst[q][r][c] = src[r][col0 + q*C + c]   (0 past the last column K)
// 8 bf16 (16 B) per thread; K, C and col0 are multiples of 8, so a chunk is all in or all out.
__global__ void __launch_bounds__(256) gather_cols_kernel(const uint4* __restrict__ src, int K8, int R, int col08,
                                                          int C8, int Q, uint4* __restrict__ dst) {
  const int64_t total = (int64_t)Q * R * C8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % C8);
    const int64_t qr = i / C8;
    const int r = (int)(qr % R), q = (int)(qr / R);
    const int col = col08 + q * C8 + c;
    dst[i] = col < K8 ? src[(int64_t)r * K8 + col] : make_uint4(0, 0, 0, 0);
  }
}

void gather_cols_bf16(const at::Tensor& src, int64_t col0, at::Tensor& dst) {
  TORCH_CHECK(src.dtype() == at::kBFloat16 && dst.dtype() == at::kBFloat16 && src.dim() == 2 && dst.dim() == 3 &&
                  src.is_contiguous() && dst.is_contiguous(), "gather_cols_bf16: src [R][K], dst [Q][R][C] bf16");
  const int64_t R = src.size(0), K = src.size(1), Q = dst.size(0), C = dst.size(2);
  TORCH_CHECK(dst.size(1) == R && K % 8 == 0 && C % 8 == 0 && col0 % 8 == 0 && col0 >= 0,
              "gather_cols_bf16: shapes (K, C, col0 must be multiples of 8)");
  const int64_t total = Q * R * (C / 8);
  if (total == 0) return;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 2048);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  gather_cols_kernel<<<grid, 256, 0, stream>>>((const uint4*)src.data_ptr(), (int)(K / 8), (int)R, (int)(col0 / 8),
                                               (int)(C / 8), (int)Q, (uint4*)dst.data_ptr());
}

}  // namespace mihvd
