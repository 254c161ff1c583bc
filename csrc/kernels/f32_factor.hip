// fp32 factor-gather plane (mihvd/parallel/factor.py): this rank's R rows of the
// summed dense/kernel gradient from the gathered fp32 factors, with their Adam update applied from
// the accumulators (dW3 never goes through HBM unless stored for a test).
//
//   g[r][n] = sum_s A[s][r] D[s][n]    A = a2 columns of this rank's rows [NB][R] (all-to-all),
//                                      D = every rank's dz [NB][1024] (all-gather), NB = N B
//
// 8 ceil(R / 16) blocks (column group = blockIdx & 7, the XCD): a block owns 16 rows x 128 columns; its 8 waves (two per SIMD) split the
// NB samples into contiguous ranges of 4-sample k steps. v_mfma_f32_16x16x4_f32 with the rows of W3
// on the MFMA row axis: lane (lr, lg) supplies A[s0 + lg][r0 + lr] and, for its 8 column tiles c,
// D[s0 + lg][n0 + 8 lr + c] (two float4 loads per k step), so C of tile c is
// g[r0 + 4 lg + i][n0 + 8 lr + c]. Operands come straight from L2 (A and D are 1.6 MB at N = 8),
// batches of 2 k steps in a ring of five register stages (four batches in flight). The eight waves'
// partial tiles meet in LDS in a fixed order (deterministic) and form the block's [16][128] tile,
// updated with coalesced float4 accesses by the same adam1() as every other optimizer kernel
// (gscale = 1/N of the Average). Replaces a library GEMM (R x NB x 1024, 11.3 us at N = 8 on MI355X) plus an adam_step
// launch over the rows.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "f32_common.h"

namespace mihvd {

constexpr int FAC_U = 2;   // k steps per load batch
constexpr int FAC_W = 8;   // waves per block (the samples split 8 ways: two waves per SIMD)
constexpr int FAC_S = 5;   // register stages of the load ring

template <bool ADAM, bool STORE>
__global__ void __launch_bounds__(512) f32_factor_rows_kernel(const float* __restrict__ A, const float* __restrict__ D,
                                                              int NB, int R, float* __restrict__ out, F32Adam ad) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  f32x4* red = reinterpret_cast<f32x4*>(smf);  // [wave][tile][lane]: 64 KB
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15,
            lg = lane >> 4;
  // XCD-aware order: the 8 column groups are the 8 XCDs (the hardware deals blocks round-robin,
  // blockIdx & 7), so every block reading a group's D columns shares one L2 (400 KB at N = 8)
  const int r0 = (blockIdx.x >> 3) * 16, n0 = (blockIdx.x & 7) * 128;
  const int ra = min(r0 + lr, R - 1);
  const bool rin = r0 + lr < R;
  const int steps = (NB + 3) / 4, per = (steps + FAC_W - 1) / FAC_W;
  const int k_lo = wave * per, k_hi = min(steps, k_lo + per);
  f32x4 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* dp = D + n0 + 8 * lr;
  struct Stage {
    float a[FAC_U];
    float4 x[FAC_U], y[FAC_U];
  };
  auto load = [&](Stage& st, int kb) {
#pragma unroll
    for (int u = 0; u < FAC_U; ++u) {
      const int s = 4 * (kb + u) + lg;
      const bool ok = kb + u < k_hi && s < NB;
      const int sc = min(s, NB - 1);
      st.a[u] = mask_f(A[(int64_t)sc * R + ra], ok && rin);
      st.x[u] = mask_f4(*reinterpret_cast<const float4*>(dp + (int64_t)sc * 1024), ok);
      st.y[u] = mask_f4(*reinterpret_cast<const float4*>(dp + (int64_t)sc * 1024 + 4), ok);
    }
  };
  auto mma = [&](const Stage& st) {
#pragma unroll
    for (int u = 0; u < FAC_U; ++u) {
      acc[0] = mfma4(st.a[u], st.x[u].x, acc[0]);
      acc[1] = mfma4(st.a[u], st.x[u].y, acc[1]);
      acc[2] = mfma4(st.a[u], st.x[u].z, acc[2]);
      acc[3] = mfma4(st.a[u], st.x[u].w, acc[3]);
      acc[4] = mfma4(st.a[u], st.y[u].x, acc[4]);
      acc[5] = mfma4(st.a[u], st.y[u].y, acc[5]);
      acc[6] = mfma4(st.a[u], st.y[u].z, acc[6]);
      acc[7] = mfma4(st.a[u], st.y[u].w, acc[7]);
    }
  };
  // ring of FAC_S register stages, FAC_S - 1 batches in flight ahead of the MFMAs (the first pass
  // over D misses the XCD's L2 on every block at once, so the lead has to cover MALL latency);
  // wave-uniform trip count; steps past k_hi load zeros, and a batch wholly past k_hi is skipped
  Stage st[FAC_S];
#pragma unroll
  for (int j = 0; j < FAC_S - 1; ++j) load(st[j], k_lo + j * FAC_U);
  for (int kb = k_lo; kb < k_hi; kb += FAC_S * FAC_U) {
#pragma unroll
    for (int j = 0; j < FAC_S; ++j) {
      load(st[(j + FAC_S - 1) % FAC_S], kb + (j + FAC_S - 1) * FAC_U);
      __builtin_amdgcn_sched_barrier(0);
      if (kb + j * FAC_U < k_hi) mma(st[j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) red[(wave * 8 + c) * 64 + lane] = acc[c];
  __syncthreads();
  // wave w finishes tile w (lane (lr, lg): rows r0 + 4 lg + i of column n0 + 8 lr + w) into a
  // [16][128] tile, which the block then streams through Adam with coalesced float4 accesses
  f32x4 g = red[(0 * 8 + wave) * 64 + lane];
#pragma unroll
  for (int q = 1; q < FAC_W; ++q) g += red[(q * 8 + wave) * 64 + lane];
  float* tile = smf + FAC_W * 8 * 64 * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) tile[(4 * lg + i) * 128 + 8 * lr + wave] = g[i];
  __syncthreads();
  const int rr = t >> 5, cc = 4 * (t & 31), r = r0 + rr;  // 512 threads x 4 = 16 x 128
  if (r < R) {
    const int64_t o = (int64_t)r * 1024 + n0 + cc;
    float4 gg = *reinterpret_cast<const float4*>(tile + rr * 128 + cc);
    if constexpr (STORE) *reinterpret_cast<float4*>(out + o) = gg;
    if constexpr (ADAM) {
      const AdamCoef coef = f32_adam_coef(ad);
      float4 pp = *reinterpret_cast<const float4*>(ad.p + o), mm = *reinterpret_cast<const float4*>(ad.m + o),
             vv = *reinterpret_cast<const float4*>(ad.v + o);
      adam4_f32(pp, mm, vv, gg, coef);
      *reinterpret_cast<float4*>(ad.p + o) = pp;
      *reinterpret_cast<float4*>(ad.m + o) = mm;
      *reinterpret_cast<float4*>(ad.v + o) = vv;
    }
  }
}
constexpr int FAC_LDS = FAC_W * 8 * 64 * 16 + 16 * 128 * 4;  // 73,728 B: partial tiles + the row tile

// ------------------------------------------------------------------------------------------ //
// Replicated factor plane (small N: mihvd/parallel/factor.py factor_gather_all_): EVERY row of the
// summed gradient from the all-gathered factors A = a2 [N][B][3136] and D = dz [N][B][1024],
//   g[f][n] = sum_q sum_b A[q][b][f] D[q][b][n]   (segments q in rank order: the same sum on every rank)
// with Adam applied from the accumulators to every row (the optimizer stays replicated: no row
// gather afterwards). The wgrad role of f32_fc1_bwd's row form without its dgrad: one block per 16
// rows of W3 (196 blocks), 8 waves of 128 columns in 8 chunks of 16; per segment the wave holds
// that segment's a2 column in registers (the MFMA B operand) and stages each dz chunk through a
// per-wave double buffer in LDS (A = dz^T, ds_read_b32 of 64 consecutive floats per MFMA:
// conflict-free); v_mfma_f32_16x16x4_f32 with two alternating accumulators per chunk as in
// f32_fc1_bwd (at N = 1 the result is bitwise that kernel's). In the last segment the chunk's Adam
// follows its MFMAs, with p / m / v loaded two chunks ahead, so W3's update streams under the MFMAs.
// ------------------------------------------------------------------------------------------ //
template <int G, int KS, bool STORE>
__global__ void __launch_bounds__(512) f32_factor_full_kernel(const float* __restrict__ A, const float* __restrict__ D,
                                                              int N, int B, float* __restrict__ out, F32Adam ad) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  static_assert(KS <= 4 * G && KS > 4 * G - 4, "K steps cover the segment's last partial group");
  constexpr int BUF = 16 * G * 16;  // floats per buffer: [16 G samples][16 columns or rows]
  constexpr int PA = 2;             // p / m / v chunks loaded ahead of their Adam
  constexpr int NS = PA + 1;        // ... in a ring of register slots
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int f0 = 16 * blockIdx.x, nb = 128 * wave;
  float* buf0 = smf + wave * 2 * BUF;  // this wave's dz chunk double buffer
  float* abuf = smf + 16 * BUF;        // the block's a2 column of a segment, [sample][16 rows], double-buffered
  const int64_t rowo = (int64_t)(f0 + lr) * 1024 + nb + 4 * lg;
  const AdamCoef coef = f32_adam_coef(ad);
  f32x4 tot[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) tot[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Operands run ahead of the MFMAs across segment boundaries: the dz chunks two ahead (two register
  // stages), the next segment's a2 column (one LDS copy per block, read by all eight waves as the
  // MFMA B operand) from chunk 4 on, p / m / v of the last segment two chunks ahead (its first two
  // during the segment before it; three ahead spilled registers). Per chunk a wave's 25 MFMAs (~800 cycles) cannot cover an
  // L2 round trip issued one chunk ahead.
  float4 zs[2][G];
  float4 pv[NS], mv[NS], vv[NS];
  auto load_z = [&](float4 (&z)[G], const float* Ds, int c) {
    const int n = nb + 16 * c + 4 * (lane & 3);
#pragma unroll
    for (int it = 0; it < G; ++it) {
      const int b = (lane >> 2) + 16 * it;
      z[it] = mask_f4(*reinterpret_cast<const float4*>(Ds + (int64_t)min(b, B - 1) * 1024 + n), b < B);
    }
  };
  // the a2 column of a segment: 16 G samples x 16 rows, 4 floats per thread (threads past it idle)
  constexpr int ANT = (16 * G * 16) / 4;
  float4 an = make_float4(0.f, 0.f, 0.f, 0.f);
  auto load_a = [&](const float* As) {
    if (t < ANT) {
      const int b = t >> 2, r4 = 4 * (t & 3);
      an = mask_f4(*reinterpret_cast<const float4*>(As + (int64_t)min(b, B - 1) * 3136 + f0 + r4), b < B);
    }
  };
  auto store_a = [&](int slot) {
    if (t < ANT) *reinterpret_cast<float4*>(abuf + slot * BUF + 4 * t) = an;
  };
  auto load_pmv = [&](int c) {
    const int64_t o = rowo + 16 * c;
    const int slot = c % NS;
    pv[slot] = *reinterpret_cast<const float4*>(ad.p + o);
    mv[slot] = *reinterpret_cast<const float4*>(ad.m + o);
    vv[slot] = *reinterpret_cast<const float4*>(ad.v + o);
  };
  load_a(A);
  load_z(zs[0], D, 0);
  load_z(zs[1], D, 1);
  if (N == 1) {
#pragma unroll
    for (int c = 0; c < PA; ++c) load_pmv(c);
  }
  store_a(0);
  __syncthreads();
  for (int seg = 0; seg < N; ++seg) {  // block-uniform
    const float* Ds = D + (int64_t)seg * B * 1024;
    const float* Dn = Ds + (int64_t)B * 1024;
    const float* as = abuf + (seg & 1) * BUF;
    const bool last = seg == N - 1, more = seg + 1 < N, next_last = seg + 2 == N;
    if (more) load_a(A + (int64_t)(seg + 1) * B * 3136);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float* buf = buf0 + (c & 1) * BUF;
#pragma unroll
      for (int it = 0; it < G; ++it) {
        const int row = (lane >> 2) + 16 * it;
        *reinterpret_cast<float4*>(buf + row * 16 + 4 * (lane & 3)) = zs[c & 1][it];
      }
      if (c + 2 < 8) load_z(zs[c & 1], Ds, c + 2);
      else if (more) load_z(zs[c & 1], Dn, c + 2 - 8);
      if (last && c + PA < 8) load_pmv(c + PA);
      if (next_last && c >= 8 - PA) load_pmv(c - (8 - PA));
      if (c == 4 && more) store_a((seg + 1) & 1);  // (the other buffer: nobody reads it this segment)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the wave's LDS writes before its reads
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      f32x4 w0 = {0.f, 0.f, 0.f, 0.f}, w1 = w0;
#pragma unroll
      for (int s = 0; s + 1 < KS; s += 2) {
        w0 = mfma4(buf[(4 * s + lg) * 16 + lr], as[(4 * s + lg) * 16 + lr], w0);
        w1 = mfma4(buf[(4 * s + 4 + lg) * 16 + lr], as[(4 * s + 4 + lg) * 16 + lr], w1);
      }
      if constexpr (KS & 1)
        w0 = mfma4(buf[(4 * (KS - 1) + lg) * 16 + lr], as[(4 * (KS - 1) + lg) * 16 + lr], w0);
      tot[c] += w0 + w1;
      if (last) {
        const f32x4 g = tot[c];
        float4 gg = make_float4(g[0], g[1], g[2], g[3]);
        const int64_t o = rowo + 16 * c;
        if constexpr (STORE) *reinterpret_cast<float4*>(out + o) = gg;
        const int slot = c % NS;
        float4 pp = pv[slot], mm = mv[slot], vq = vv[slot];
        adam4_f32(pp, mm, vq, gg, coef);
        *reinterpret_cast<float4*>(ad.p + o) = pp;
        *reinterpret_cast<float4*>(ad.m + o) = mm;
        *reinterpret_cast<float4*>(ad.v + o) = vq;
      }
    }
    if (more) __syncthreads();  // the next a2 column is in LDS; every wave is done with this one
  }
}
constexpr int ffu_lds(int G) { return (8 * 2 + 2) * 16 * G * 16 * 4; }  // G = 7: 129,024 B

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
  const dim3 grid((unsigned)(8 * ((R + 15) / 16)));
  auto stream = c10::hip::getCurrentHIPStream().stream();
  float* op = store ? out->data_ptr<float>() : nullptr;
  auto launch = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, FAC_LDS);
    kern<<<grid, 64 * FAC_W, FAC_LDS, stream>>>(a2c.data_ptr<float>(), dz.data_ptr<float>(), (int)NB, (int)R, op, ad);
  };
  if (adam && store) launch(f32_factor_rows_kernel<true, true>);
  else if (adam) launch(f32_factor_rows_kernel<true, false>);
  else launch(f32_factor_rows_kernel<false, true>);
}

// Every row of dW3 over the N B all-gathered samples (segments of B, rank order) with Adam on
// every row: a2 [N B][3136], dz [N B][1024], p / m / v the full dense/kernel [3136][1024]; out
// (optional): the gradient.
void f32_factor_full(const at::Tensor& a2, const at::Tensor& dz, int64_t B, const c10::optional<at::Tensor>& out,
                     at::Tensor& p, at::Tensor& m, at::Tensor& v, const at::Tensor& state, double lr, double beta1,
                     double beta2, double eps, double grad_scale, int64_t rule) {
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_factor_full: batch 1..128");
  TORCH_CHECK(dz.dim() >= 2 && dz.size(-1) == 1024 && dz.numel() % (B * 1024) == 0, "f32_factor_full: dz [N B][1024]");
  const int64_t N = dz.numel() / (B * 1024);
  TORCH_CHECK(N >= 1 && N <= 64, "f32_factor_full: 1..64 segments");
  fac_chk(dz, N * B * 1024, "f32_factor_full: dz");
  fac_chk(a2, N * B * 3136, "f32_factor_full: a2");
  fac_chk(p, 3136 * 1024, "f32_factor_full: p");
  fac_chk(m, 3136 * 1024, "f32_factor_full: m");
  fac_chk(v, 3136 * 1024, "f32_factor_full: v");
  TORCH_CHECK(state.is_cuda() && state.dtype() == at::kLong && state.numel() >= ST_WORDS, "f32_factor_full: state");
  const bool store = out.has_value() && out->defined();
  if (store) fac_chk(*out, 3136 * 1024, "f32_factor_full: out");
  F32Adam ad;
  ad.p = p.data_ptr<float>();
  ad.m = m.data_ptr<float>();
  ad.v = v.data_ptr<float>();
  ad.state = state.data_ptr<int64_t>();
  ad.lr = (float)lr;
  ad.b1 = (float)beta1;
  ad.b2 = (float)beta2;
  ad.eps = (float)eps;
  ad.gscale = (float)grad_scale;
  ad.rule = (int)rule;
  float* op = store ? out->data_ptr<float>() : nullptr;
  const int G = (int)((B + 15) / 16);
  auto stream = c10::hip::getCurrentHIPStream().stream();
  auto launch = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, ffu_lds(G));
    kern<<<196, 512, ffu_lds(G), stream>>>(a2.data_ptr<float>(), dz.data_ptr<float>(), (int)N, (int)B, op, ad);
  };
  // the exact K steps of the headline batch (B = 97..100: 25), as f32_fc1_bwd
  if (G == 7 && (B + 3) / 4 == 25) {
    if (store) launch(f32_factor_full_kernel<7, 25, true>);
    else launch(f32_factor_full_kernel<7, 25, false>);
    return;
  }
#define FFU_CASE(GG)                                                  \
  case GG:                                                            \
    if (store) launch(f32_factor_full_kernel<GG, 4 * GG, true>);      \
    else launch(f32_factor_full_kernel<GG, 4 * GG, false>);           \
    break;
  switch (G) {
    FFU_CASE(1)
    FFU_CASE(2)
    FFU_CASE(3)
    FFU_CASE(4)
    FFU_CASE(5)
    FFU_CASE(6)
    FFU_CASE(7)
    default:
      FFU_CASE(8)
  }
#undef FFU_CASE
}

}  // namespace mihvd
