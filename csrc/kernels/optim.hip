// Fused optimizer over the flat fp32 parameter buffer (K12/K13 of SURVEY.md §2.5).
//
// One pass reads (p, m, v, g) and writes (p, m, v) plus the bf16 shadow of p that the MFMA
// forward/backward kernels consume, so no separate cast kernel runs per step. The gradient scale
// (1/size for Average, fused here instead of a separate division) and the TF1 Adam rule
// (horovod/tensorflow_mnist.py:130):
//     lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t);  p -= lr_t * m / (sqrt(v) + eps)
// With a device step-state tensor the step t is read on the device (graph-replayable) and the
// forward step counter is advanced by block 0. An optional device loss-scale pair [scale, found]
// (dp_kernels.hip) makes the update skip itself after an overflow and divides by the scale.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include <hip/hip_fp16.h>

#include "common.h"

namespace mihvd {

__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, u16* __restrict__ shadow,
                                                   int64_t n4, int64_t* __restrict__ state, int64_t host_t, float lr,
                                                   float b1, float b2, float eps, float gscale, int rule, int bump,
                                                   const float* __restrict__ ls) {
  if (bump && state && blockIdx.x == 0 && threadIdx.x == 0) state[ST_FWD] += 1;
  if (ls) {  // dynamic loss scaling (dp_kernels.hip): skip on overflow, unscale fused into gscale
    if (ls[1] != 0.f) return;
    gscale /= ls[0];
  }
  const AdamCoef c = adam_coef((float)(state ? state[ST_OPT] : host_t), lr, b1, b2, eps, gscale, rule);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    const uint2 sh = adam4(pp, mm, vv, gg, c);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (shadow) reinterpret_cast<uint2*>(shadow)[i] = sh;
  }
}

__global__ void __launch_bounds__(256) scale_cast_kernel(const float* __restrict__ src, u16* __restrict__ dst, int64_t n4,
                                                         float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 s = reinterpret_cast<const float4*>(src)[i];
    reinterpret_cast<uint2*>(dst)[i] = make_uint2((uint32_t)f2bf(s.x * scale) | ((uint32_t)f2bf(s.y * scale) << 16),
                                                  (uint32_t)f2bf(s.z * scale) | ((uint32_t)f2bf(s.w * scale) << 16));
  }
}

__global__ void __launch_bounds__(256) bf16_to_f32_kernel(const u16* __restrict__ src, float* __restrict__ dst, int64_t n4,
                                                          float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const uint2 s = reinterpret_cast<const uint2*>(src)[i];
    reinterpret_cast<float4*>(dst)[i] = make_float4(bf2f((u16)(s.x & 0xffff)) * scale, bf2f((u16)(s.x >> 16)) * scale,
                                                    bf2f((u16)(s.y & 0xffff)) * scale, bf2f((u16)(s.y >> 16)) * scale);
  }
}

// fp16 wire format of Compression.fp16 (the same pack/unpack with scale as the bf16 pair above).
__global__ void __launch_bounds__(256) scale_cast_f16_kernel(const float* __restrict__ src, __half* __restrict__ dst,
                                                             int64_t n4, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 s = reinterpret_cast<const float4*>(src)[i];
    __half2* d = reinterpret_cast<__half2*>(dst) + 2 * i;
    d[0] = __floats2half2_rn(s.x * scale, s.y * scale);
    d[1] = __floats2half2_rn(s.z * scale, s.w * scale);
  }
}

__global__ void __launch_bounds__(256) f16_to_f32_kernel(const __half* __restrict__ src, float* __restrict__ dst,
                                                         int64_t n4, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const __half2* s = reinterpret_cast<const __half2*>(src) + 2 * i;
    const float2 a = __half22float2(s[0]), b = __half22float2(s[1]);
    reinterpret_cast<float4*>(dst)[i] = make_float4(a.x * scale, a.y * scale, b.x * scale, b.y * scale);
  }
}

static int grid_for(int64_t n4) {
  int64_t g = (n4 + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 2048));
}

void adam_step(at::Tensor& p, const at::Tensor& g, at::Tensor& m, at::Tensor& v, const c10::optional<at::Tensor>& shadow,
               const c10::optional<at::Tensor>& state, int64_t host_step, double lr, double b1, double b2, double eps,
               double grad_scale, int64_t rule, int64_t bump, const c10::optional<at::Tensor>& loss_scale,
               int64_t max_blocks) {
  const int64_t n = p.numel();
  TORCH_CHECK(p.dtype() == at::kFloat && g.dtype() == at::kFloat && m.dtype() == at::kFloat && v.dtype() == at::kFloat,
              "adam_step: fp32 buffers expected");
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam_step: size mismatch");
  TORCH_CHECK(n % 4 == 0, "adam_step: flat buffer length must be a multiple of 4");
  TORCH_CHECK(p.is_contiguous() && g.is_contiguous() && m.is_contiguous() && v.is_contiguous(), "adam_step: contiguous");
  u16* sp = nullptr;
  if (shadow.has_value() && shadow->defined()) {
    TORCH_CHECK(shadow->dtype() == at::kBFloat16 && shadow->numel() == n, "adam_step: shadow must be bf16 like p");
    sp = (u16*)shadow->data_ptr();
  }
  int64_t* st = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  TORCH_CHECK(st != nullptr || host_step >= 1, "adam_step: step must be >= 1");
  const float* ls = nullptr;
  if (loss_scale.has_value() && loss_scale->defined()) {
    TORCH_CHECK(loss_scale->dtype() == at::kFloat && loss_scale->numel() == 2, "adam_step: loss_scale is float32 [2]");
    ls = loss_scale->data_ptr<float>();
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  // max_blocks > 0 caps the grid (grid-stride loop): a capped update sharing the GPU with
  // another stream's kernels leaves CUs to them instead of queueing thousands of blocks ahead.
  int grid = grid_for(n / 4);
  if (max_blocks > 0) grid = std::min<int>(grid, (int)max_blocks);
  adam_kernel<<<grid, 256, 0, stream>>>(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                                                   v.data_ptr<float>(), sp, n / 4, st, host_step, (float)lr, (float)b1,
                                                   (float)b2, (float)eps, (float)grad_scale, (int)rule, (int)bump, ls);
}

void scale_cast_bf16(const at::Tensor& src, at::Tensor& dst, double scale) {
  TORCH_CHECK(src.dtype() == at::kFloat && dst.dtype() == at::kBFloat16 && src.numel() == dst.numel() && src.numel() % 4 == 0,
              "scale_cast_bf16");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  scale_cast_kernel<<<grid_for(src.numel() / 4), 256, 0, stream>>>(src.data_ptr<float>(), (u16*)dst.data_ptr(),
                                                                   src.numel() / 4, (float)scale);
}

void bf16_to_f32(const at::Tensor& src, at::Tensor& dst, double scale) {
  TORCH_CHECK(src.dtype() == at::kBFloat16 && dst.dtype() == at::kFloat && src.numel() == dst.numel() && src.numel() % 4 == 0,
              "bf16_to_f32");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  bf16_to_f32_kernel<<<grid_for(src.numel() / 4), 256, 0, stream>>>((const u16*)src.data_ptr(), dst.data_ptr<float>(),
                                                                     src.numel() / 4, (float)scale);
}

void scale_cast_f16(const at::Tensor& src, at::Tensor& dst, double scale) {
  TORCH_CHECK(src.dtype() == at::kFloat && dst.dtype() == at::kHalf && src.numel() == dst.numel() && src.numel() % 4 == 0,
              "scale_cast_f16");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  scale_cast_f16_kernel<<<grid_for(src.numel() / 4), 256, 0, stream>>>(src.data_ptr<float>(), (__half*)dst.data_ptr(),
                                                                       src.numel() / 4, (float)scale);
}

void f16_to_f32(const at::Tensor& src, at::Tensor& dst, double scale) {
  TORCH_CHECK(src.dtype() == at::kHalf && dst.dtype() == at::kFloat && src.numel() == dst.numel() && src.numel() % 4 == 0,
              "f16_to_f32");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  f16_to_f32_kernel<<<grid_for(src.numel() / 4), 256, 0, stream>>>((const __half*)src.data_ptr(), dst.data_ptr<float>(),
                                                                   src.numel() / 4, (float)scale);
}

}  // namespace mihvd
