// fp32 factor-gather plane (mihvd/parallel/factor.py): this rank's R rows of the
// summed dense/kernel gradient from the gathered fp32 factors, with their Adam update applied from
// the accumulators (dW3 never goes through HBM unless stored for a test).
//
//   g[r][n] = sum_s A[s][r] D[s][n]    A = a2 columns of this rank's rows [NB][R] (all-to-all),
//                                      D = every rank's dz [NB][1024] (all-gather), NB = N B
//
// grid (ceil(R / 16), 8): a block owns 16 rows x 128 columns; its 4 waves (one per SIMD) split the
// NB samples into contiguous ranges of 4-sample k steps. v_mfma_f32_16x16x4_f32 with the rows of W3
// on the MFMA row axis: lane (lr, lg) supplies A[s0 + lg][r0 + lr] and, for its 8 column tiles c,
// D[s0 + lg][n0 + 8 lr + c] (two float4 loads per k step), so C of tile c is
// g[r0 + 4 lg + i][n0 + 8 lr + c]. Operands come straight from L2 (A and D are 1.6 MB at N = 8),
// batches of 4 k steps loaded one batch ahead. The four waves' partial tiles meet in LDS in a fixed
// order (deterministic); wave w then finishes tiles 2w, 2w + 1: a lane holds 2 consecutive columns
// of 4 rows, updated with the same adam1() as every other optimizer kernel (gscale = 1/N of the
// Average). Replaces a library GEMM (R x NB x 1024, 11.3 us at N = 8 on MI355X) plus an adam_step
// launch over the rows.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "f32_common.h"

namespace mihvd {

constexpr int FAC_U = 4;  // k steps per load batch

template <bool ADAM, bool STORE>
__global__ void __launch_bounds__(256) f32_factor_rows_kernel(const float* __restrict__ A, const float* __restrict__ D,
                                                              int NB, int R, float* __restrict__ out, F32Adam ad) {
  __shared__ f32x4 red[4 * 8 * 64];  // [wave][tile][lane]: 32 KB
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15,
            lg = lane >> 4;
  const int r0 = blockIdx.x * 16, n0 = blockIdx.y * 128;
  const int ra = min(r0 + lr, R - 1);
  const bool rin = r0 + lr < R;
  const int steps = (NB + 3) / 4, per = (steps + 3) / 4;
  const int k_lo = wave * per, k_hi = min(steps, k_lo + per);
  f32x4 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* dp = D + n0 + 8 * lr;
  float a0[FAC_U], a1[FAC_U];
  float4 d00[FAC_U], d01[FAC_U], d10[FAC_U], d11[FAC_U];
  auto load = [&](float (&a)[FAC_U], float4 (&x)[FAC_U], float4 (&y)[FAC_U], int kb) {
#pragma unroll
    for (int u = 0; u < FAC_U; ++u) {
      const int s = 4 * (kb + u) + lg;
      const bool ok = kb + u < k_hi && s < NB;
      const int sc = min(s, NB - 1);
      a[u] = mask_f(A[(int64_t)sc * R + ra], ok && rin);
      x[u] = mask_f4(*reinterpret_cast<const float4*>(dp + (int64_t)sc * 1024), ok);
      y[u] = mask_f4(*reinterpret_cast<const float4*>(dp + (int64_t)sc * 1024 + 4), ok);
    }
  };
  auto mma = [&](const float (&a)[FAC_U], const float4 (&x)[FAC_U], const float4 (&y)[FAC_U]) {
#pragma unroll
    for (int u = 0; u < FAC_U; ++u) {
      acc[0] = mfma4(a[u], x[u].x, acc[0]);
      acc[1] = mfma4(a[u], x[u].y, acc[1]);
      acc[2] = mfma4(a[u], x[u].z, acc[2]);
      acc[3] = mfma4(a[u], x[u].w, acc[3]);
      acc[4] = mfma4(a[u], y[u].x, acc[4]);
      acc[5] = mfma4(a[u], y[u].y, acc[5]);
      acc[6] = mfma4(a[u], y[u].z, acc[6]);
      acc[7] = mfma4(a[u], y[u].w, acc[7]);
    }
  };
  // ping-pong over two register sets: batch b + 1 in flight while batch b's MFMAs issue (wave-uniform
  // trip count; steps past k_hi load zeros and add exact zeros)
  load(a0, d00, d01, k_lo);
  for (int kb = k_lo; kb < k_hi; kb += 2 * FAC_U) {
    load(a1, d10, d11, kb + FAC_U);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, d00, d01);
    __builtin_amdgcn_sched_barrier(0);
    if (kb + 2 * FAC_U < k_hi) load(a0, d00, d01, kb + 2 * FAC_U);
    __builtin_amdgcn_sched_barrier(0);
    if (kb + FAC_U < k_hi) mma(a1, d10, d11);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) red[(wave * 8 + c) * 64 + lane] = acc[c];
  __syncthreads();
  f32x4 g[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = 2 * wave + h;
    g[h] = (red[(0 * 8 + c) * 64 + lane] + red[(1 * 8 + c) * 64 + lane]) +
           (red[(2 * 8 + c) * 64 + lane] + red[(3 * 8 + c) * 64 + lane]);
  }
  AdamCoef coef{};
  if constexpr (ADAM) coef = f32_adam_coef(ad);
  const int n = n0 + 8 * lr + 2 * wave;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + 4 * lg + i;
    if (r >= R) break;
    const int64_t o = (int64_t)r * 1024 + n;
    float2 gg = make_float2(g[0][i], g[1][i]);
    if constexpr (STORE) *reinterpret_cast<float2*>(out + o) = gg;
    if constexpr (ADAM) {
      float2 pp = *reinterpret_cast<const float2*>(ad.p + o), mm = *reinterpret_cast<const float2*>(ad.m + o),
             vv = *reinterpret_cast<const float2*>(ad.v + o);
      adam1(pp.x, mm.x, vv.x, gg.x, coef);
      adam1(pp.y, mm.y, vv.y, gg.y, coef);
      *reinterpret_cast<float2*>(ad.p + o) = pp;
      *reinterpret_cast<float2*>(ad.m + o) = mm;
      *reinterpret_cast<float2*>(ad.v + o) = vv;
    }
  }
}

static void fac_chk(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous() && t.numel() == numel &&
                  ((uintptr_t)t.data_ptr() & 15) == 0,
              what, ": expected a 16-byte aligned contiguous fp32 CUDA tensor of ", numel, " elements");
}

// g rows = a2c^T dz over all samples; with p/m/v/state: Adam on the rows (W3 rows of this rank,
// [R][1024]) from the accumulators; out (optional): the gradient rows.
void f32_factor_rows(const at::Tensor& a2c, const at::Tensor& dz, const c10::optional<at::Tensor>& out,
                     const c10::optional<at::Tensor>& p, const c10::optional<at::Tensor>& m,
                     const c10::optional<at::Tensor>& v, const c10::optional<at::Tensor>& state, double lr,
                     double beta1, double beta2, double eps, double grad_scale, int64_t rule) {
  TORCH_CHECK(dz.dim() >= 2 && dz.size(-1) == 1024, "f32_factor_rows: dz [NB][1024]");
  const int64_t NB = dz.numel() / 1024;
  TORCH_CHECK(NB >= 1 && a2c.numel() % NB == 0, "f32_factor_rows: a2c [NB][R]");
  const int64_t R = a2c.numel() / NB;
  TORCH_CHECK(R >= 1 && R <= 3136, "f32_factor_rows: 1..3136 rows");
  fac_chk(dz, NB * 1024, "f32_factor_rows: dz");
  TORCH_CHECK(a2c.is_cuda() && a2c.dtype() == at::kFloat && a2c.is_contiguous(), "f32_factor_rows: a2c");
  const bool store = out.has_value() && out->defined();
  if (store) fac_chk(*out, R * 1024, "f32_factor_rows: out");
  F32Adam ad;
  const bool adam = p.has_value() && p->defined();
  if (adam) {
    TORCH_CHECK(m.has_value() && m->defined() && v.has_value() && v->defined() && state.has_value() &&
                    state->defined(), "f32_factor_rows: Adam needs p, m, v and the step state");
    fac_chk(*p, R * 1024, "f32_factor_rows: p");
    fac_chk(*m, R * 1024, "f32_factor_rows: m");
    fac_chk(*v, R * 1024, "f32_factor_rows: v");
    ad.p = p->data_ptr<float>();
    ad.m = m->data_ptr<float>();
    ad.v = v->data_ptr<float>();
    ad.state = state->data_ptr<int64_t>();
    ad.lr = (float)lr;
    ad.b1 = (float)beta1;
    ad.b2 = (float)beta2;
    ad.eps = (float)eps;
    ad.gscale = (float)grad_scale;
    ad.rule = (int)rule;
  }
  TORCH_CHECK(adam || store, "f32_factor_rows: nothing to write (neither out nor the Adam operands)");
  const dim3 grid((unsigned)((R + 15) / 16), 8);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  float* op = store ? out->data_ptr<float>() : nullptr;
  if (adam && store)
    f32_factor_rows_kernel<true, true><<<grid, 256, 0, stream>>>(a2c.data_ptr<float>(), dz.data_ptr<float>(), (int)NB,
                                                                 (int)R, op, ad);
  else if (adam)
    f32_factor_rows_kernel<true, false><<<grid, 256, 0, stream>>>(a2c.data_ptr<float>(), dz.data_ptr<float>(),
                                                                  (int)NB, (int)R, op, ad);
  else
    f32_factor_rows_kernel<false, true><<<grid, 256, 0, stream>>>(a2c.data_ptr<float>(), dz.data_ptr<float>(),
                                                                  (int)NB, (int)R, op, ad);
}

}  // namespace mihvd
