// Exact-fp32 backward kernels of the MNIST CNN (see f32_fwd.hip for the precision contract).
//
//   f32_fc1_bwd      one launch, three block roles:
//                      dgrad: g2 = (dz W3^T) * [a2 > 0], routed through the pool argmax idx2 into
//                             the full conv2 output gradient dY2 [B][14][14][64] (every element
//                             written: value or zero), + per-block db2 partial rows
//                      small: db3, dW4, db4
//                      wgrad: dW3 = a2^T dz in 64x64 tiles              [MFMA 16x16x4 / 32x32x2]
//   f32_conv2_bwd    one launch, two block roles:
//                      dgrad: dA1 = dY2 (x) W2 (implicit GEMM, K = 25 taps x 64) over 16-pixel
//                             tiles of the batch; conv1's pooled-ReLU mask; the conv1 weight
//                             gradient of those pixels from the routed gradient (sparse: one 5x5
//                             x-patch per pooled element) -> per-block partial rows
//                      wgrad: dW2 partial slabs per (kernel row, 32-channel half, image group)
//                                                                           [MFMA 16x16x4 / 32x32x2]
//   f32_conv_reduce  dW2 = sum of slabs; dW1, db1, db2 = sums of the partial rows (fixed order:
//                    deterministic, no atomics)
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "f32_common.h"

namespace mihvd {

// Phase stamps (study instrument, off unless f32_stamps_enable set the buffer): thread 0 of each
// block of f32_conv2_bwd records the shader clock (s_memtime) at its phase boundaries into
// stamps[block][16] with vector stores (slots 8..15: each wave's end of the dgrad tap loop).
// Compiled in only by a study build (MIHVD_F32_STAMPS=1 at build time, mihvd/_build.py): each stamp
// loads the buffer pointer from a __device__ variable and waits for it (s_waitcnt vmcnt(0)), which
// costs a dependent L2 round trip at every phase boundary of the production kernel.
__device__ unsigned long long* g_c2b_stamps = nullptr;
__device__ __forceinline__ void c2b_stamp(int k) {
#ifdef MIHVD_F32_STAMPS
  unsigned long long* p = g_c2b_stamps;
  if (p != nullptr && threadIdx.x == 0) p[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memtime();
#endif
}
// f32_fc1_bwd row form (f32_stamps_enable kernel 2): 0 start, 1 + c: wave 0's end of chunk c,
// 9: after the partial-exchange barrier, 10: end of the routing epilogue (wave 0)
__device__ unsigned long long* g_f1r_stamps = nullptr;
__device__ __forceinline__ void f1r_stamp(int k) {
#ifdef MIHVD_F32_STAMPS
  unsigned long long* p = g_f1r_stamps;
  if (p != nullptr && threadIdx.x == 0) p[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memtime();
#endif
}
// per-wave stamp (lane 0 of every wave): slot 8 + wave
__device__ __forceinline__ void c2b_stamp_wave() {
#ifdef MIHVD_F32_STAMPS
  unsigned long long* p = g_c2b_stamps;
  if (p != nullptr && (threadIdx.x & 63) == 0) p[blockIdx.x * 16 + 8 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_memtime();
#endif
}

// ------------------------------------------------------------------------------------------ //
// f32_fc1_bwd
// ------------------------------------------------------------------------------------------ //
constexpr int F1B_SMALL = 33;  // blocks of the small reductions (db3, dW4, db4) behind the row blocks

// ------------------------------------------------------------------------------------------ //
// f32_fc1_bwd, row form: one block per 16 rows of W3 (= 16 channels of one pooling
// window), 8 waves; wave w owns the 128 columns n in [128 w, 128 w + 128) of those rows, in 8
// chunks of 16. Per chunk the wave holds p = W3[f0 + lr][n .. n + 3] (4 consecutive columns per
// lane: lane group lg -> n = nn + 4 lg) and uses it twice:
//   dgrad  g2[b][f] += sum_n W3[f][n] dz[b][n]  (K-split over the waves; p is the K-contiguous A
//          operand, dz[b][n..n+3] from LDS the B operand; G sample tiles = G accumulators)
//   wgrad  dW3[f][n] = sum_b a2[b][f] dz[b][n]  (16x16x4, C[row = n][col = f]: the lane's four
//          accumulator rows are exactly the four columns of p it holds; A = dz^T from LDS, B = the
//          block's a2 column held in registers for the whole kernel)
// and then, with ADAM (world size 1: dW3 is final here), applies Adam to those four elements from
// the accumulators: W3 is read ONCE per step for dgrad, gradient and update, and dW3 never goes
// through HBM (STORE keeps it in the gradient buffer: N > 1, where it is reduced first, and tests).
// dz chunks ([B][16] per wave, rows >= B zero) are staged through a per-wave double buffer in LDS
// (row stride 16 floats: the b32 reads of the wgrad operand are conflict-free) by register loads
// issued one chunk ahead; p/m/v are loaded two chunks ahead. The eight dgrad partials meet in LDS
// in a fixed order (deterministic) and the routing epilogue writes dY2 and the db2 partial rows.
// ------------------------------------------------------------------------------------------ //
constexpr int F1R_BLOCKS = 196;                       // 3136 / 16 rows
constexpr int F1R_LDS_BUF = F32_MAXB * 16;            // floats per wave buffer
constexpr int F1R_LDS = 8 * 2 * F1R_LDS_BUF * 4;      // 131,072 B
static_assert(8 * 8 * 64 * 16 <= F1R_LDS, "fc1 row form: dgrad partial exchange fits the dz buffers");

// fc1 row form: the dz chunk swizzle (see store_z) and the column position of element `col` of `row`
__device__ __forceinline__ int f1r_swz(int row) { return ((row >> 3) & 1) << 1; }
__device__ __forceinline__ int f1r_col(int row, int col) { return 4 * ((col >> 2) ^ f1r_swz(row)) + (col & 3); }

__device__ __forceinline__ void lds_wave_fence() {
  // the wave's own LDS writes before its later reads (LDS executes one wave's ops in order); a
  // compiler barrier keeps the program order
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Small reductions over the batch for 512-thread blocks: db3 (16 blocks), dW4 (16 blocks), db4.
__device__ __forceinline__ void f32_fc1_small512(int bid, const float* __restrict__ dz, const float* __restrict__ h,
                                                 const float* __restrict__ dlog, float* __restrict__ gb3,
                                                 float* __restrict__ gW4, float* __restrict__ gb4, int B, float* smf) {
  const int t = threadIdx.x, nn = t & 63, rg = t >> 6;  // 8 row groups of 16 samples
  if (bid < 16) {
    const int n = bid * 64 + nn;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int b = rg * 16 + i;
      s += mask_f(dz[(int64_t)min(b, B - 1) * 1024 + n], b < B);
    }
    smf[rg * 64 + nn] = s;
    __syncthreads();
    if (t < 64)
      gb3[n] = ((smf[nn] + smf[64 + nn]) + (smf[128 + nn] + smf[192 + nn])) +
               ((smf[256 + nn] + smf[320 + nn]) + (smf[384 + nn] + smf[448 + nn]));
    return;
  }
  if (bid < 32) {
    const int r = bid - 16, n = r * 64 + nn;
    float* dls = smf;                  // [128][10]
    float* red = smf + F32_MAXB * 10;  // [8][64][10]
    float hv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int b = rg * 16 + i;
      hv[i] = mask_f(h[(int64_t)min(b, B - 1) * 1024 + n], b < B);
    }
    for (int i = t; i < F32_MAXB * 10; i += 512) dls[i] = i < B * 10 ? dlog[i] : 0.f;
    __syncthreads();
    float s[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) s[c] = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int c = 0; c < 10; ++c) s[c] = fmaf(hv[i], dls[(rg * 16 + i) * 10 + c], s[c]);
#pragma unroll
    for (int c = 0; c < 10; ++c) red[(rg * 64 + nn) * 10 + c] = s[c];
    __syncthreads();
    for (int i = t; i < 640; i += 512) {
      const int n2 = i / 10, c = i - n2 * 10;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; q += 2) v += red[(q * 64 + n2) * 10 + c] + red[((q + 1) * 64 + n2) * 10 + c];
      gW4[(r * 64 + n2) * 10 + c] = v;
    }
    return;
  }
  // db4: thread = (class c, row group of 3)
  const int c = t % 10, gq = t / 10;
  float s = 0.f;
  if (gq < 43) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int b = gq * 3 + i;
      s += mask_f(dlog[min(b, B - 1) * 10 + c], b < B);
    }
  }
  smf[t] = s;
  __syncthreads();
  if (t < 10) {
    float tot = 0.f;
    for (int q = 0; q < 43; ++q) tot += smf[q * 10 + t];
    gb4[t] = tot;
  }
}

// The next step's batch gathered ahead (resident set): the images into xpre [B][784] and the labels
// into ypre [B], by the small-reduction blocks, which run on CUs the 196 row blocks leave free and
// finish long before them; conv1 and the head of the next step read these with one load instead of
// the counter -> rows -> image / label chain. (In the head, a step earlier in the chain, the same
// gather cost 0.2 us of head time: profiles/r06/roofline_f32_gather_ahead_r06x.md.)
struct F32Prefetch {
  const float* x = nullptr;        // the resident set [n_pool][784]
  const int64_t* labels = nullptr; // [n_pool]
  const int* rows = nullptr;       // the epoch order [n_pool]
  const int64_t* state = nullptr;  // state[ST_FWD]: this step (the next is + 1)
  int n_pool = 0;
  float* xpre = nullptr;
  int* ypre = nullptr;
};

__device__ __forceinline__ void f32_prefetch_next(const F32Prefetch& pf, int s, int nsb, int B) {
  const int t = threadIdx.x;
  const int64_t step = pf.state[ST_FWD] + 1;
  for (int b = s; b < B; b += nsb) {  // block-uniform
    const int row = pf.rows[(int)((step * (int64_t)B + b) % pf.n_pool)];
    if (t < 196)
      reinterpret_cast<float4*>(pf.xpre + (int64_t)b * 784)[t] = reinterpret_cast<const float4*>(pf.x + (int64_t)row * 784)[t];
    else if (t == 196)
      pf.ypre[b] = (int)pf.labels[row];
  }
}

// p/m/v are loaded two chunks ahead (PD, a ring of three register slots; four ahead measured no
// faster: 28.2 vs 27.8 us, profiles/r04/kbench_f32_r04e.txt). Pinning the dgrad MFMA order with
// sched_barrier measured slower (+2 us, r04).
// KW: K steps of the wgrad chain, 4 samples each: 4 G (the padded tiles) by default, ceil(B / 4) in
// the exact-batch instantiation (B = 100: 25 instead of 28 MFMAs per chunk; the rows past the
// batch are zero either way).
template <int G, bool ADAM, bool STORE, int KW = 4 * G>
__global__ void __launch_bounds__(512) f32_fc1_bwd_rows_kernel(
    const float* __restrict__ dz, const float* __restrict__ a2, const uint8_t* __restrict__ idx2,
    const float* __restrict__ h, const float* __restrict__ dlog, float* __restrict__ w3, float* __restrict__ dY2,
    float* __restrict__ db2p, float* __restrict__ gW3, float* __restrict__ gb3, float* __restrict__ gW4,
    float* __restrict__ gb4, int B, F32Adam ad, F32Prefetch pf) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int bid = blockIdx.x;
  if (bid >= F1R_BLOCKS) {
    if (pf.ypre != nullptr) f32_prefetch_next(pf, bid - F1R_BLOCKS, F1B_SMALL, B);
    f32_fc1_small512(bid - F1R_BLOCKS, dz, h, dlog, gb3, gW4, gb4, B, smf);
    return;
  }
  constexpr int KS = KW;  // K steps of the wgrad chain
  constexpr int PD = 2;
  // dgrad only (neither the fused Adam nor the stored gradient: the fp32 factor-gather plane forms
  // dW3 from every rank's factors elsewhere): no a2 operand, no wgrad MFMAs, W3 read once
  constexpr bool WG = ADAM || STORE;
  static_assert(KS <= 4 * G && KS > 4 * G - 4, "wgrad K steps cover the batch tiles' last partial group");
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int f0 = 16 * bid, nb = 128 * wave;
  f1r_stamp(0);
  // the routing epilogue's a2 / idx2 operands (they depend on the block alone) are loaded at the
  // start, so the epilogue after the exchange does not begin with a dependent global round trip
  // (r05h: 27.98 -> 27.03 us)
  const int jt = bid >> 2, co_e = 16 * (bid & 3) + 4 * (lane >> 4), j_e = 64 * jt + co_e;
  const int m_e = 16 * (t >> 6) + (lane & 15), mc_e = min(m_e, B - 1);
  float4 av_e = make_float4(0.f, 0.f, 0.f, 0.f);
  uint32_t ix_e = 0u;
  auto load_route = [&]() {
    if (t < G * 64) {
      av_e = *reinterpret_cast<const float4*>(a2 + (int64_t)mc_e * 3136 + j_e);
      ix_e = *reinterpret_cast<const uint32_t*>(idx2 + (int64_t)mc_e * 3136 + j_e);
    }
  };
  float* buf0 = smf + wave * 2 * F1R_LDS_BUF;
  // the wgrad B operand for the whole kernel: a2[4 s + lg][f0 + lr] (zero past the batch)
  float a2r[KS];
  auto load_a2r = [&]() {
    if constexpr (WG) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int b = 4 * s + lg;
        a2r[s] = mask_f(a2[(int64_t)min(b, B - 1) * 3136 + f0 + lr], b < B);
      }
    }
  };
  // dz staging: chunk c = dz[0 .. 16 G)[nb + 16 c .. + 16): lane -> row (lane >> 2) + 16 it, float4 (lane & 3)
  float4 zst[G];
  auto load_z = [&](int c) {
    const int n = nb + 16 * c + 4 * (lane & 3);
#pragma unroll
    for (int it = 0; it < G; ++it) {
      const int b = (lane >> 2) + 16 * it;
      zst[it] = mask_f4(*reinterpret_cast<const float4*>(dz + (int64_t)min(b, B - 1) * 1024 + n), b < B);
    }
  };
  // dz rows in LDS with the 16-byte chunks of rows 8..15 (mod 16) XOR-swizzled by 2: the dgrad's
  // ds_read_b128 (lane (lr, lg) -> row lr, chunk lg) then hits 16 distinct slots per 16-lane group
  // (2-way conflicts without), and the wgrad's ds_read_b32 of two adjacent rows stays conflict-free
  auto store_z = [&](float* buf) {
#pragma unroll
    for (int it = 0; it < G; ++it) {
      const int row = (lane >> 2) + 16 * it;
      *reinterpret_cast<float4*>(buf + row * 16 + 4 * ((lane & 3) ^ f1r_swz(row))) = zst[it];
    }
  };
  // p (and m, v) of chunk c: W3[f0 + lr][nb + 16 c + 4 lg .. + 3]
  const int64_t rowo = (int64_t)(f0 + lr) * 1024 + nb + 4 * lg;
  constexpr int NS = PD + 1;
  float4 pv[NS], mv[NS], vv[NS];
  auto load_pmv = [&](int c, int slot) {
    const int64_t o = rowo + 16 * c;
    pv[slot] = *reinterpret_cast<const float4*>(w3 + o);
    if constexpr (ADAM) {
      mv[slot] = *reinterpret_cast<const float4*>(ad.m + o);
      vv[slot] = *reinterpret_cast<const float4*>(ad.v + o);
    }
  };
  AdamCoef coef{};
  if constexpr (ADAM) coef = f32_adam_coef(ad);
  f32x4 acc[G];
#pragma unroll
  for (int u = 0; u < G; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the first chunk's dz and p / m / v first: its LDS stores and dgrad MFMAs (in-order vmcnt) then
  // wait for those alone, not for the 25 a2 loads of the wgrad operand and the routing operands
  // issued behind them (pinned: the scheduler hoisted the a2 loads to the top; fc1_bwd 28.7 -> 28.1 us
  // under rocprofv3, profiles/r05/fc1_bwd_load_order_r05ab.txt)
  load_z(0);
  load_pmv(0, 0);
  __builtin_amdgcn_sched_barrier(0);
  load_a2r();
  load_route();
#pragma unroll
  for (int c = 1; c < PD; ++c) load_pmv(c, c);
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float* buf = buf0 + (c & 1) * F1R_LDS_BUF;
    store_z(buf);
    if (c + 1 < 8) load_z(c + 1);
    if (c + PD < 8) load_pmv(c + PD, (c + PD) % NS);
    lds_wave_fence();
    const int s3 = c % NS;
    const float4 p = pv[s3];
    // dgrad: G tiles of 16 samples, the four k elements of the chunk outer (independent accumulators)
    float4 zb[G];
#pragma unroll
    for (int u = 0; u < G; ++u) zb[u] = *reinterpret_cast<const float4*>(buf + (16 * u + lr) * 16 + 4 * (lg ^ f1r_swz(lr)));
#pragma unroll
    for (int u = 0; u < G; ++u) acc[u] = mfma4(p.x, zb[u].x, acc[u]);
#pragma unroll
    for (int u = 0; u < G; ++u) acc[u] = mfma4(p.y, zb[u].y, acc[u]);
#pragma unroll
    for (int u = 0; u < G; ++u) acc[u] = mfma4(p.z, zb[u].z, acc[u]);
#pragma unroll
    for (int u = 0; u < G; ++u) acc[u] = mfma4(p.w, zb[u].w, acc[u]);
    // wgrad: dW3[f0 + lr][nn + 4 lg + i] over the batch, two alternating accumulators. (Reading every
    // LDS operand of the chunk ahead of its MFMAs with the order pinned by sched_barrier, and four
    // wgrad chains, was measured slower: 33.6 vs 27.7 us with the fused Adam, 27.5 vs 22.9 without,
    // profiles/r04/kbench_f32_r04g.txt; the pinned order keeps the global loads and the Adam VALU
    // work from interleaving with the MFMAs)
    if constexpr (!WG) {
      f1r_stamp(1 + c);
      continue;
    }
    f32x4 w0 = {0.f, 0.f, 0.f, 0.f}, w1 = w0;
#pragma unroll
    for (int s = 0; s + 1 < KS; s += 2) {
      const float z0 = buf[(4 * s + lg) * 16 + f1r_col(4 * s + lg, lr)];
      const float z1 = buf[(4 * s + 4 + lg) * 16 + f1r_col(4 * s + 4 + lg, lr)];
      w0 = mfma4(z0, a2r[s], w0);
      w1 = mfma4(z1, a2r[s + 1], w1);
    }
    if constexpr (KS & 1) w0 = mfma4(buf[(4 * (KS - 1) + lg) * 16 + f1r_col(4 * (KS - 1) + lg, lr)], a2r[KS - 1], w0);
    const f32x4 g = w0 + w1;
    const int64_t o = rowo + 16 * c;
    float4 gg = make_float4(g[0], g[1], g[2], g[3]);
    if constexpr (STORE) *reinterpret_cast<float4*>(gW3 + o) = gg;
    if constexpr (ADAM) {
      float4 pp = p, mm = mv[s3], vq = vv[s3];
      adam4_f32(pp, mm, vq, gg, coef);
      *reinterpret_cast<float4*>(w3 + o) = pp;
      *reinterpret_cast<float4*>(ad.m + o) = mm;
      *reinterpret_cast<float4*>(ad.v + o) = vq;
    }
    f1r_stamp(1 + c);
  }
  // the eight K-part partials meet in LDS (the dz buffers are dead after the barrier)
  __syncthreads();
  f1r_stamp(9);
  float4* red = reinterpret_cast<float4*>(smf);  // [8 waves][8 tiles][64 lanes]
#pragma unroll
  for (int u = 0; u < G; ++u) red[(wave * 8 + u) * 64 + lane] = make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
  __syncthreads();
  const int py = jt / 7, px = jt - 7 * py;
  if (t < G * 64) {  // wave u handles tile u
    const int u = t >> 6, ln = lane, r = ln & 15;
    float4 s = red[(0 * 8 + u) * 64 + ln];
#pragma unroll
    for (int w = 1; w < 8; ++w) s = f4add(s, red[(w * 8 + u) * 64 + ln]);
    const float sv[4] = {s.x, s.y, s.z, s.w};
    const int m = m_e, co = co_e;
    const bool valid = m < B;
    const float4 av = av_e;
    const uint32_t ix = ix_e;
    const float ae[4] = {av.x, av.y, av.z, av.w};
    float gq[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) gq[e] = (valid && ae[e] > 0.f) ? sv[e] : 0.f;
    float sm[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) sm[e] = row_sum16(gq[e]);  // over the 16 samples of tile u
    if (r == 0)
      *reinterpret_cast<float4*>(db2p + ((int64_t)u * 49 + jt) * 64 + co) = make_float4(sm[0], sm[1], sm[2], sm[3]);
    if (valid) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float o4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o4[e] = (int)((ix >> (8 * e)) & 0xff) == d ? gq[e] : 0.f;
        const int y = 2 * py + (d >> 1), x = 2 * px + (d & 1);
        *reinterpret_cast<float4*>(dY2 + (((int64_t)m * 14 + y) * 14 + x) * 64 + co) =
            make_float4(o4[0], o4[1], o4[2], o4[3]);
      }
    }
  }
  f1r_stamp(10);
}

// ------------------------------------------------------------------------------------------ //
// f32_conv2_bwd (512-thread blocks)
// ------------------------------------------------------------------------------------------ //
// Tall padded dY2 image: rows of CBF_RWD pixels (18 used: 2 + 14 + 2 padding columns) of CBF_PS
// floats (64 channels + padding). 72 x 22 makes every ds_read_b128 of the tap loop conflict-free:
// each 16-lane group (two 4-channel chunks x 8 consecutive output pixels) lands on 16 distinct
// 16-byte slots for every tap and every row/image wrap of a tile (scripts/ldssim_conv2.py: 1.00
// LDS cycles per group, against 2.70 for the 68 x 18 layout of round 3).
constexpr int CBF_PS = 72, CBF_RWD = 22, CBF_RS = CBF_RWD * CBF_PS, CBF_MAXR = 16;
constexpr int CBF_IMG = CBF_MAXR * CBF_RS;            // floats: tall padded dY2 rows
// one-round form (two tap-loop passes per dgrad block, twice the tiles): rows of up to 10 tiles
constexpr int CBF_MAXR2 = 21, CBF_IMG2 = CBF_MAXR2 * CBF_RS;
constexpr int cbf_maxr(int npass) { return npass == 2 ? CBF_MAXR2 : CBF_MAXR; }
constexpr int cbf_img(int npass) { return cbf_maxr(npass) * CBF_RS; }
// padded x images [32][34]: the epilogue's 16 lanes of one pixel read its x patch at the pooled
// argmax position (channel-dependent: offsets 0, 1, row, row + 1), so a 32-float row put the 0 and
// row offsets on one bank (2-way ds_read_b32 conflicts, PMC ~5e5 cycles per launch); 34 separates them
constexpr int CBF_XS = 34, CBF_XIMG = 32 * CBF_XS;
constexpr int CBF_XIM = 2 * CBF_XIMG;                 // two padded x images
constexpr int CBF_PW = 8 * 2 * 64 * 4;                // per-wave conv1 partials (8 waves x 26 x 16 used)
// The x images and the conv1 partials live in the dead image area behind the co-quarter partial
// exchange (written after the tap loops' barrier): the image alone sets the dgrad LDS size.
constexpr int cbf_red(int tpb) { return 4 * 2 * tpb * 64 * 4; }           // floats of the exchange
constexpr int CBF_LDS_DG = CBF_IMG * 4;                                     // 101,376 B
constexpr int CBF_A1S = 14 * 18 * 32, CBF_DYS = 196 * 32, CBF_WBUF = CBF_A1S + CBF_DYS;
constexpr int CBF_LDS_WG = 2 * CBF_WBUF * 4;                                // 114,688 B
constexpr int CBF_LDS = CBF_LDS_DG > CBF_LDS_WG ? CBF_LDS_DG : CBF_LDS_WG;
constexpr int CBF_LDS_DG2 = CBF_IMG2 * 4;                                   // 133,056 B
constexpr int CBF_LDS2 = CBF_LDS_DG2 > CBF_LDS_WG ? CBF_LDS_DG2 : CBF_LDS_WG;
constexpr int CBF_IG = 4;                                                   // images per wgrad block
constexpr int CBF_IG2 = 8;                                                  // ... in the one-round form
constexpr int CP_F32 = 832;                                                 // [dW1 (800) | db1 (32)]
static_assert(CBF_LDS <= 163840 && CBF_LDS2 <= 163840, "f32_conv2_bwd LDS");
static_assert(cbf_red(10) + CBF_XIM + CBF_PW <= CBF_IMG2, "one-round dgrad exchange + x images + partials fit");
static_assert(8 * 26 * 16 <= CBF_PW, "the VALU conv1-wgrad epilogue's partials fit");
static_assert(cbf_red(7) + CBF_XIM + CBF_PW <= CBF_IMG, "dgrad exchange + x images + partials fit the image");
static_assert(4 * 5 * 4 * 64 * 16 <= CBF_LDS_WG, "wgrad partial exchange fits the staging buffers");

// dgrad role. Pixels of the batch (flattened [B][196], raster order) in 16-pixel tiles; block owns
// tiles [bid TPB, (bid+1) TPB). dA1[p][ci] = sum_{tap, co} dY2pad[p + (4 - kh, 4 - kw)][co] W2[tap][ci][co]:
// A = the routed gradient (tall padded image rows in LDS, co contiguous -> float4), B = the W2 tap
// slice read as [ci][co] (co contiguous -> float4): a wave's whole B (25 taps x 16 co x 16 ci =
// 100 floats per lane) is loaded into registers once, so the tap loop has no global load and no
// barrier. 8 waves: wave w = ci half (w & 1) x co
// quarter (w >> 1) of K; the four co-quarter partials are summed through LDS before the epilogue.
// A block barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt(0)), not for
// its global loads in flight — __syncthreads() also drains vmcnt, which would make a register
// prefetch issued before it (the W2 operand) complete before the barrier. The asm memory clobbers
// keep the compiler from moving LDS accesses across it (s_barrier alone is not a memory fence).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef __attribute__((address_space(3))) void lds_void_t;

// The W2 register operand is loaded BEFORE the staging barrier (after the staging loads, so the
// staging writes wait only for their own loads), and the barrier orders LDS alone: the 25 W2 loads
// per lane (200 KB per block from L2) land while the dY2 image is staged instead of after it. (The
// conv1 weight gradient of the epilogue on MFMA instead of VALU measured slower every time it was
// tried: dgrad role 42.3 -> 45.7 us, profiles/r05/conv2_bwd_mfma_epilogue_r05y.txt; removed.)
// NPASS = 2 (the one-round form): TPB tiles in two tap-loop passes of TPB / 2 over the same
// register-resident W2 (the A register sets are reused, the accumulators of both passes live on),
// so a block loads W2 once for twice the tiles and the halo rows are staged once for both.
// FRAG: W2 from the fragment copy (f32_w2_frag_block in f32_fwd.hip): one contiguous 1 KB per wave
// and tap instead of 16 scattered 64-byte row pieces.
template <int TPB, int NPASS = 1, bool FRAG = false>
__device__ __forceinline__ void f32_conv2_dgrad_block(
    int bid, const float* __restrict__ dY2, const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ idx1, const float* __restrict__ x, const int* __restrict__ rows, int n_pool,
    const int64_t* __restrict__ state, float* __restrict__ cpart, int B, float* smf, const float* __restrict__ w2f) {
  static_assert(TPB % NPASS == 0, "tiles split evenly over the passes");
  constexpr int TP = TPB / NPASS;                                        // tiles per pass
  constexpr int MAXCH = (cbf_maxr(NPASS) * 18 * 16 + 511) / 512;         // dY2 chunks per thread
  float* dimg = smf;
  float* xim = smf + cbf_red(TPB);  // behind the partial exchange, written after the tap loops
  float* pw = xim + CBF_XIM;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int np = 196 * B, T0 = bid * TPB;
  const int P0 = 16 * T0, P1 = min(16 * (T0 + TPB), np) - 1;
  const int b0 = P0 / 196, b1i = P1 / 196;
  const int R0 = 18 * b0 + (P0 - 196 * b0) / 14, R1 = 18 * b1i + (P1 - 196 * b1i) / 14 + 5;
  const int nch = (R1 - R0) * 288;  // 18 pixels x 16 float4
  const int nt = wave & 1, cq = wave >> 1;
  // the dataset rows of the block's (at most two) images: block-uniform, so the step counter and
  // the two row indices are scalar loads whose waits leave the vector loads below in flight
  int xrow0 = b0, xrow1 = min(b0 + 1, B - 1);
  if (rows != nullptr) {
    const int64_t step = state ? state[ST_FWD] : 0;
    xrow0 = rows[(int)((step * (int64_t)B + xrow0) % n_pool)];
    xrow1 = rows[(int)((step * (int64_t)B + xrow1) % n_pool)];
  }
  // 1. loads: the first two taps' weight fragments, the dY2 rows, the (at most two) x images
  float4 iv[MAXCH];
#pragma unroll
  for (int it = 0; it < MAXCH; ++it) {
    const int i = min(t + 512 * it, nch - 1);
    const int rr = i / 288, rem = i - rr * 288, c = rem >> 4, ch = rem & 15;
    const int R = R0 + rr, bb = R / 18, y = R - 18 * bb - 2, xx = c - 2;
    const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
    const float4 v = *reinterpret_cast<const float4*>(
        dY2 + (((int64_t)bb * 14 + (in ? y : 0)) * 14 + (in ? xx : 0)) * 64 + ch * 4);
    iv[it] = mask_f4(v, in);
  }
#pragma unroll
  for (int it = 0; it < MAXCH; ++it) {
    const int i = t + 512 * it;
    if (i < nch) {
      const int rr = i / 288, rem = i - rr * 288;
      *reinterpret_cast<float4*>(dimg + (rr * CBF_RWD + (rem >> 4)) * CBF_PS + (rem & 15) * 4) = iv[it];
    }
  }
  // this wave's whole B operand in registers: wb[tap] = W2[tap][16 nt + lr][16 cq + 4 lg .. + 3],
  // issued right behind the staging writes (which wait only for the staging loads), so they are in
  // flight across the barrier
  const float* wq = w2 + (16 * nt + lr) * 64 + 16 * cq + 4 * lg;
  const float4* wfq = reinterpret_cast<const float4*>(w2f) + wave * 25 * 64 + lane;
  float4 wb[25];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int tap = 0; tap < 25; ++tap) wb[tap] = FRAG ? wfq[tap * 64] : *reinterpret_cast<const float4*>(wq + tap * 2048);
  __builtin_amdgcn_sched_barrier(0);
  int abase[TPB];
#pragma unroll
  for (int i = 0; i < TPB; ++i) {
    const int P = min(16 * (T0 + i) + lr, np - 1);
    const int bb = P / 196, p = P - 196 * bb, py = p / 14, px = p - 14 * py;
    abase[i] = ((18 * bb + py - R0) * CBF_RWD + px) * CBF_PS + 16 * cq + 4 * lg;
  }
  f32x4 acc[TPB];
#pragma unroll
  for (int i = 0; i < TPB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  lds_barrier();  // the dY2 image is complete; the W2 loads stay in flight
  c2b_stamp(1);
  // the epilogue's conv1 operands (ReLU sign and pool argmax of this lane's a1 elements), prefetched:
  // (nt, tile) pairs p = wave + 8k, lane pixel 4 lg + r
  constexpr int NP = (2 * TPB + 7) / 8;
  float ea[NP][4];
  int ex[NP][4];
  auto load_epi = [&]() {
#pragma unroll
    for (int k = 0; k < NP; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pp = wave + 8 * k;
        const int P = 16 * (T0 + (pp >> 1)) + 4 * lg + r;
        const bool ok = pp < 2 * TPB && P < np;
        const int64_t o = (int64_t)min(P, np - 1) * 32 + 16 * nt + lr;
        ea[k][r] = mask_f(a1[o], ok);
        ex[k][r] = idx1[o];
      }
  };
  load_epi();
  // the x patches are needed only by the epilogue: loaded here, they land during the tap loop. The
  // rows of the block's (at most two) images were looked up at block start with block-uniform
  // (scalar) loads, so no vector wait on that dependent chain drains the W2 / epilogue loads
  float xv[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = t + 512 * it, pix = i & 1023, Y = (pix >> 5) - 2, X = (pix & 31) - 2;
    const int row = it < 2 ? xrow0 : xrow1;  // i >> 10 == it >> 1 (512-thread blocks)
    const bool in = Y >= 0 && Y < 28 && X >= 0 && X < 28;
    xv[it] = mask_f(x[(int64_t)row * 784 + (in ? Y * 28 + X : 0)], in);
  }
  // Software pipeline, fully unrolled: the A chunks of tap t + 1 are read into the other register
  // set before tap t's MFMAs issue; sched_barrier pins that order (left alone, the scheduler
  // reuses one register set and waits on each read right before its MFMAs).
  float4 ra[TP], rb[TP];
  auto run_pass = [&](auto i0c) {
    constexpr int I0 = decltype(i0c)::value;  // first tile of the pass
    auto load_a = [&](float4 (&a)[TP], int tap) {
      const int kh = tap / 5, kw = tap - 5 * kh;
      const int aoff = ((4 - kh) * CBF_RWD + (4 - kw)) * CBF_PS;
#pragma unroll
      for (int i = 0; i < TP; ++i) a[i] = *reinterpret_cast<const float4*>(dimg + abase[I0 + i] + aoff);
    };
    auto mfma_tap = [&](const float4 (&a)[TP], const float4& w) {
      // k-element j outer, tiles inner: consecutive MFMAs use different accumulators
#pragma unroll
      for (int i = 0; i < TP; ++i) acc[I0 + i] = mfma4(a[i].x, w.x, acc[I0 + i]);
#pragma unroll
      for (int i = 0; i < TP; ++i) acc[I0 + i] = mfma4(a[i].y, w.y, acc[I0 + i]);
#pragma unroll
      for (int i = 0; i < TP; ++i) acc[I0 + i] = mfma4(a[i].z, w.z, acc[I0 + i]);
#pragma unroll
      for (int i = 0; i < TP; ++i) acc[I0 + i] = mfma4(a[i].w, w.w, acc[I0 + i]);
    };
    load_a(ra, 0);
#pragma unroll
    for (int tap = 0; tap < 25; tap += 2) {
      if (tap + 1 < 25) load_a(rb, tap + 1);
      __builtin_amdgcn_sched_barrier(0);
      mfma_tap(ra, wb[tap]);
      __builtin_amdgcn_sched_barrier(0);
      if (tap + 1 < 25) {
        if (tap + 2 < 25) load_a(ra, tap + 2);
        __builtin_amdgcn_sched_barrier(0);
        mfma_tap(rb, wb[tap + 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  run_pass(std::integral_constant<int, 0>{});
  if constexpr (NPASS == 2) run_pass(std::integral_constant<int, TP>{});
  c2b_stamp(2);
  c2b_stamp_wave();
  __syncthreads();  // every wave is done with the dY2 image
  c2b_stamp(7);
#pragma unroll
  for (int it = 0; it < 4; ++it) {  // (complete after the next barrier)
    const int i = t + 512 * it, sl = i >> 10, pix = i & 1023;
    xim[sl * CBF_XIMG + (pix >> 5) * CBF_XS + (pix & 31)] = xv[it];
  }
  // 2. sum the four co-quarter partials (the dY2 image is dead now)
  f32x4* red = reinterpret_cast<f32x4*>(dimg);  // [cq][nt][TPB][64]
#pragma unroll
  for (int i = 0; i < TPB; ++i) red[((cq * 2 + nt) * TPB + i) * 64 + lane] = acc[i];
  __syncthreads();
  // 3. epilogue: (nt, tile) pairs p = wave, wave + 8, ...: mask -> g1, the conv1 weight gradient of
  //    the routed g1 (one 5x5 patch of x per pooled element), db1
  float s25[26];
#pragma unroll
  for (int e = 0; e < 26; ++e) s25[e] = 0.f;
  const int ci = 16 * nt + lr;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int p = wave + 8 * k;  // wave-uniform; p & 1 == nt
    if (p >= 2 * TPB) break;
    const int i = p >> 1;
    const f32x4 sum = ((red[((0 * 2 + nt) * TPB + i) * 64 + lane] + red[((1 * 2 + nt) * TPB + i) * 64 + lane]) +
                       red[((2 * 2 + nt) * TPB + i) * 64 + lane]) +
                      red[((3 * 2 + nt) * TPB + i) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int P = 16 * (T0 + i) + 4 * lg + r;
      if (P < np) {
        const int bb = P / 196, pp = P - 196 * bb, py = pp / 14, px = pp - 14 * py;
        const float g = ea[k][r] > 0.f ? sum[r] : 0.f;
        const int ix = ex[k][r];
        const float* xs = xim + (bb - b0) * CBF_XIMG + (2 * py + (ix >> 1)) * CBF_XS + 2 * px + (ix & 1);
#pragma unroll
        for (int kh = 0; kh < 5; ++kh)
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) s25[kh * 5 + kw] = fmaf(g, xs[kh * CBF_XS + kw], s25[kh * 5 + kw]);
        s25[25] += g;
      }
    }
  }
  // 4. sum over the four lane groups (same channel), then over the four waves of each ci half
#pragma unroll
  for (int e = 0; e < 26; ++e) {
    float v = s25[e];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    s25[e] = v;
  }
  if (lg == 0) {
#pragma unroll
    for (int e = 0; e < 26; ++e) pw[(wave * 26 + e) * 16 + lr] = s25[e];
  }
  __syncthreads();
  for (int q = t; q < CP_F32; q += 512) {
    const int e = q >> 5, c = q & 31, h = c >> 4, l = c & 15;
    const float v = (pw[((h + 0) * 26 + e) * 16 + l] + pw[((h + 2) * 26 + e) * 16 + l]) +
                    (pw[((h + 4) * 26 + e) * 16 + l] + pw[((h + 6) * 26 + e) * 16 + l]);
    cpart[(int64_t)bid * CP_F32 + q] = v;  // q = tap * 32 + ci (dW1, HWIO) or 800 + ci (db1)
  }
  c2b_stamp(3);
}

// wgrad role: dW2[kh][kw][ci][co] over the images of one group, kernel row kh and output-channel
// half ch. M = 32 co (A = dY2[q][co], the MFMA row axis, so a lane's four accumulator rows are a
// float4 of the HWIO slab), N = 32 ci per kw (five accumulator tiles), K = pixels q (two per MFMA).
// Every operand read is a ds_read_b32 of 32 consecutive floats (conflict-free, no padding).
// Per image: a1 padded rows kh..kh+13 [14][18][32] and the dY2 channel half [196][32], register-
// staged double buffering (the next image's loads are in flight while this one is multiplied).
// 8 waves split the K steps (w, w + 8, ...); their partial tiles are summed through LDS.
// (xcd_contiguous: f32_common.h)
__device__ __forceinline__ void f32_conv2_wgrad_block(int bid, const float* __restrict__ dY2,
                                                      const float* __restrict__ a1, float* __restrict__ slab, int B,
                                                      int ig, float* smf,
                                                      const float* __restrict__ zeros) {
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), l32 = lane & 31, hh = lane >> 5;
  const int grp = bid / 10, rem = bid - 10 * grp, kh = rem >> 1, ch = rem & 1;
  const int img0 = ig * grp, nimg = min(ig, B - img0);
  // The next image goes global -> LDS by global_load_lds_dwordx4 issued at the image start (the
  // staging image is lane-linear per wave: chunk t + 512 it at 16 (t + 512 it) bytes), so no register
  // staging and no store sits between the MFMAs; padding chunks read a zero line. The image-end
  // barrier (__syncthreads: vmcnt(0)) retires them before the buffer is read. Without the zero line
  // (`zeros` null) the register-staged form: its LDS stores one chunk per K step over steps 4..10.
  // (r05j: the role 38.96 -> 38.44 us, the step 117.73 -> 116.89 us; the other store placements
  // measured slower and were removed)
  const bool dma = zeros != nullptr;
  // this thread's seven chunk offsets within an image, computed once (per image only the image
  // term is added): chunk i < 2016 is an a1 chunk of the padded rows kh..kh+13, the rest dY2 chunks
  int loff[7];
  bool lin[7], la1[7];
#pragma unroll
  for (int it = 0; it < 7; ++it) {
    const int i = t + 512 * it;  // < 3584 = 2016 a1 chunks + 1568 dY2 chunks
    if (i < 2016) {
      const int ly = i / 144, r2 = i - 144 * ly, c = r2 >> 3, q4 = r2 & 7;
      const int y = ly + kh - 2, xx = c - 2;
      const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
      loff[it] = ((in ? y : 0) * 14 + (in ? xx : 0)) * 32 + 4 * q4;
      lin[it] = in;
      la1[it] = true;
    } else {
      const int j = i - 2016, q = j >> 3, q4 = j & 7;
      loff[it] = q * 64 + 32 * ch + 4 * q4;
      lin[it] = true;
      la1[it] = false;
    }
  }
  auto load_img = [&](int b, float4 (&v)[7]) {
    const float* pa = a1 + (int64_t)b * 6272;  // [14][14][32]
    const float* pd = dY2 + (int64_t)b * 12544;  // [196][64]
#pragma unroll
    for (int it = 0; it < 7; ++it)
      v[it] = mask_f4(*reinterpret_cast<const float4*>((la1[it] ? pa : pd) + loff[it]), lin[it]);
  };
  auto dma_img = [&](int b, float* buf) {
    const float* pa = a1 + (int64_t)b * 6272;
    const float* pd = dY2 + (int64_t)b * 12544;
    const int w64 = (t >> 6) * 64;  // this wave's first chunk: the LDS base is wave-uniform
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const float* src = lin[it] ? (la1[it] ? pa : pd) + loff[it] : zeros;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void_t*)(buf + 4 * (w64 + 512 * it)), 16, 0, 0);
    }
  };
  auto store_img = [&](float* buf, const float4 (&v)[7]) {
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const int i = t + 512 * it;
      // a1 chunk i -> A1s[(ly*18 + c)*32 + 4 q4] = buf + 4 i; dY2 chunk j -> DYs[q*32 + 4 q4] = buf + A1S + 4 j
      *reinterpret_cast<float4*>(buf + 4 * i) = v[it];
    }
  };
  f32x16 acc[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  // (loading the next image a whole image ahead instead — issued right after the previous store —
  // was measured slower: 41.3 vs 39.8 us for the role, profiles/r04/kbench_f32_r04q.txt)
  float4 v[7];
  load_img(img0, v);
  c2b_stamp(4);
  store_img(smf, v);
  __syncthreads();
  for (int n = 0; n < nimg; ++n) {
    const float* buf = smf + (n & 1) * CBF_WBUF;
    if (dma) {
      if (n + 1 < nimg) dma_img(img0 + n + 1, smf + ((n + 1) & 1) * CBF_WBUF);
    } else if (n + 1 < nimg) {
      load_img(img0 + n + 1, v);
    }
    const float* A1s = buf;
    const float* DYs = buf + CBF_A1S;
    // K steps s = wave + 8u (pixels 2s: lanes 0-31, 2s + 1: lanes 32-63). Software pipeline, fully
    // unrolled: the six LDS operands of step u + 1 are read before step u's five MFMAs issue
    // (sched_barrier pins it; left alone, the scheduler reads each operand pair right before its
    // MFMAs and waits lgkmcnt(0) every two MFMAs, which idled the MFMA pipe about half the time).
    float opa[2], opb[2][5];
    auto load_step = [&](int u, float& a, float (&b)[5]) {
      const int st = wave + 8 * u, q = 2 * st + hh, qy = q / 14, qx = q - 14 * qy;
      a = DYs[q * 32 + l32];
      const float* bp = A1s + (qy * 18 + qx) * 32 + l32;
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) b[kw] = bp[kw * 32];
    };
    // register-staged form: the next image's LDS stores are spread over this image's steps (the other
    // buffer is free since the last barrier), so the store pass overlaps MFMAs and each image ends
    // with the barrier alone
    const bool nxt = n + 1 < nimg && !dma;
    load_step(0, opa[0], opb[0]);
#pragma unroll
    for (int u = 0; u < 13; ++u) {
      const int cur = u & 1;
      if (u + 1 < 12 || (u + 1 == 12 && wave + 96 < 98)) load_step(u + 1, opa[cur ^ 1], opb[cur ^ 1]);
      __builtin_amdgcn_sched_barrier(0);
      if (u < 12 || wave + 96 < 98) {  // wave-uniform (98 = 12 x 8 + 2)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) acc[kw] = mfma32(opa[cur], opb[cur][kw], acc[kw]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // one chunk per step over u = 4..10, so each store waits only for its own load (the loads
      // return in issue order; vmcnt counts down) instead of all seven at once
      if (u >= 4 && u < 11 && nxt) {
        const int it = u - 4;
        *reinterpret_cast<float4*>(smf + ((n + 1) & 1) * CBF_WBUF + 4 * (t + 512 * it)) = v[it];
      }
    }
    __syncthreads();
    if (n < 8) c2b_stamp(8 + n);  // (study build: wgrad blocks use the per-wave slots for per-image ends)
  }
  c2b_stamp(5);
  // partial exchange: [slot][kw][g][lane] float4, two rounds (waves 4-7 -> 0-3, then 0-3 -> all)
  float4* xr = reinterpret_cast<float4*>(smf);
  if (wave >= 4) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        xr[(((wave - 4) * 5 + kw) * 4 + g) * 64 + lane] =
            make_float4(acc[kw][4 * g], acc[kw][4 * g + 1], acc[kw][4 * g + 2], acc[kw][4 * g + 3]);
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 o = xr[((wave * 5 + kw) * 4 + g) * 64 + lane];
        acc[kw][4 * g] += o.x;
        acc[kw][4 * g + 1] += o.y;
        acc[kw][4 * g + 2] += o.z;
        acc[kw][4 * g + 3] += o.w;
      }
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        xr[((wave * 5 + kw) * 4 + g) * 64 + lane] =
            make_float4(acc[kw][4 * g], acc[kw][4 * g + 1], acc[kw][4 * g + 2], acc[kw][4 * g + 3]);
  }
  __syncthreads();
  for (int it = t; it < 1280; it += 512) {
    const int kw = it >> 8, g = (it >> 6) & 3, ln = it & 63;
    const float4 a = xr[((0 * 5 + kw) * 4 + g) * 64 + ln], b = xr[((1 * 5 + kw) * 4 + g) * 64 + ln];
    const float4 c = xr[((2 * 5 + kw) * 4 + g) * 64 + ln], d = xr[((3 * 5 + kw) * 4 + g) * 64 + ln];
    const float4 s = make_float4((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                                 (a.w + b.w) + (c.w + d.w));
    const int tap = kh * 5 + kw, ci = ln & 31, co = 32 * ch + 8 * g + 4 * (ln >> 5);
    *reinterpret_cast<float4*>(slab + (int64_t)grp * 51200 + (tap * 32 + ci) * 64 + co) = s;
  }
  c2b_stamp(6);
}

// ------------------------------------------------------------------------------------------ //
// dgrad role on split-bf16 products (f32_common.h: NPROD part products per 32-deep k chunk on
// v_mfma_f32_16x16x32_bf16). The k chunk is (tap, 32 output channels): A = the routed gradient's
// three bf16 planes in LDS ([plane][tall row][18 cols][64 co]: 128 B per pixel and plane; the
// 16-byte chunk k of a pixel at k ^ x6d_swz, conflict-free for every tap and row / image wrap of a
// tile by the bank model of scripts/ldssim_conv2.py), B = W2[tap][ci][co 8 g .. + 7] (32 contiguous
// bytes of the HWIO tensor per lane), split in registers one tap ahead. 8 waves = co half (w & 1) x
// tap quarter (w >> 1: taps 0-6 | 7-12 | 13-18 | 19-24; a SIMD's two waves w, w + 4 hold quarters
// q, q + 2); each wave computes both 16-channel ci groups, so every A read feeds 2 NPROD MFMAs. The
// co halves meet first (h0 + h1), then the four quarters in the native form's order and layout, and
// the epilogue (ReLU / pool routing, the conv1 weight gradient, db1) is the native form's.
constexpr int X6D_PS = 32;                               // dwords per pixel and plane
constexpr int X6D_MAXR = 21;                             // tall rows of a 10-tile block across an image edge
constexpr int X6D_PLANE = X6D_MAXR * 18 * X6D_PS;        // dwords per plane
constexpr int X6D_LDS = 3 * X6D_PLANE * 4;               // 145,152 B
static_assert(X6D_LDS <= 163840, "split dgrad LDS");
static_assert(cbf_red(10) + CBF_XIM + CBF_PW <= 3 * X6D_PLANE, "split dgrad exchange + x images + partials fit");
__device__ __forceinline__ int x6d_swz(int pix, int r) { return (((pix >> 1) + 2 * r) & 3) << 1; }

template <int TPB, int NPROD>
__device__ __forceinline__ void f32x_conv2_dgrad_block(
    int bid, const float* __restrict__ dY2, const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ idx1, const float* __restrict__ x, const int* __restrict__ rows, int n_pool,
    const int64_t* __restrict__ state, float* __restrict__ cpart, int B, float* smf) {
  constexpr int MAXCH = (X6D_MAXR * 288 + 511) / 512;  // dY2 float4 chunks per thread
  uint32_t* img = reinterpret_cast<uint32_t*>(smf);
  float* xim = smf + cbf_red(TPB);  // behind the partial exchange, written after the tap loop
  float* pw = xim + CBF_XIM;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  // wave = ci group (w & 1) x co half (w >> 1 & 1) x tap half (w >> 2: taps 0-12 | 13-24; the two
  // waves of a SIMD, w and w + 4, hold the two halves)
  const int cg = wave & 1, h = (wave >> 1) & 1, th = wave >> 2, kp = wave >> 1;  // K part = (th, h)
  const int tap0 = th ? 13 : 0, ntap = th ? 12 : 13;
  const int np = 196 * B, T0 = bid * TPB;
  const int P0 = 16 * T0, P1 = min(16 * (T0 + TPB), np) - 1;
  const int b0 = P0 / 196, b1i = P1 / 196;
  const int R0 = 18 * b0 + (P0 - 196 * b0) / 14, R1 = 18 * b1i + (P1 - 196 * b1i) / 14 + 5;
  const int nch = (R1 - R0) * 288;  // 18 pixels x 16 float4
  int xrow0 = b0, xrow1 = min(b0 + 1, B - 1);
  if (rows != nullptr) {
    const int64_t step = state ? state[ST_FWD] : 0;
    xrow0 = rows[(int)((step * (int64_t)B + xrow0) % n_pool)];
    xrow1 = rows[(int)((step * (int64_t)B + xrow1) % n_pool)];
  }
  // B operand of a tap: W2[tap][16 cg + lr][32 h + 8 lg + j], j < 8
  const float* wq = w2 + (16 * cg + lr) * 64 + 32 * h + 8 * lg;
  float4 wraw[2];
  auto load_w = [&](int tap) {
    wraw[0] = *reinterpret_cast<const float4*>(wq + tap * 2048);
    wraw[1] = *reinterpret_cast<const float4*>(wq + tap * 2048 + 4);
  };
  load_w(tap0);
  // 1. the routed gradient rows -> the three planes
  {
    float4 iv[MAXCH];
#pragma unroll
    for (int it = 0; it < MAXCH; ++it) {
      const int i = min(t + 512 * it, nch - 1);
      const int rr = i / 288, rem = i - rr * 288, c = rem >> 4, ch = rem & 15;
      const int R = R0 + rr, bb = R / 18, y = R - 18 * bb - 2, xx = c - 2;
      const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
      const float4 v = *reinterpret_cast<const float4*>(
          dY2 + (((int64_t)bb * 14 + (in ? y : 0)) * 14 + (in ? xx : 0)) * 64 + ch * 4);
      iv[it] = mask_f4(v, in);
    }
#pragma unroll
    for (int it = 0; it < MAXCH; ++it) {
      const int i = t + 512 * it;
      if (i < nch) {
        const int rr = i / 288, rem = i - rr * 288, c = rem >> 4, ch = rem & 15;
        const int pix = rr * 18 + c;
        const int o = pix * X6D_PS + 4 * ((ch >> 1) ^ x6d_swz(pix, rr)) + 2 * (ch & 1);
        uint2 hh, mm, ll;
        x9_split4(iv[it], hh, mm, ll);
        *reinterpret_cast<uint2*>(img + o) = hh;
        *reinterpret_cast<uint2*>(img + X6D_PLANE + o) = mm;
        *reinterpret_cast<uint2*>(img + 2 * X6D_PLANE + o) = ll;
      }
    }
  }
  float xv[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = t + 512 * it, pix = i & 1023, Y = (pix >> 5) - 2, X = (pix & 31) - 2;
    const int row = it < 2 ? xrow0 : xrow1;
    const bool in = Y >= 0 && Y < 28 && X >= 0 && X < 28;
    xv[it] = mask_f(x[(int64_t)row * 784 + (in ? Y * 28 + X : 0)], in);
  }
  f32x4 acc[TPB];
#pragma unroll
  for (int i = 0; i < TPB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // the planes are complete
  // the lane's output pixel of every tile: (tall row << 16) | pixel index (row * 18 + column)
  int pb[TPB];
#pragma unroll
  for (int i = 0; i < TPB; ++i) {
    const int P = min(16 * (T0 + i) + lr, np - 1);
    const int bb = P / 196, pp = P - 196 * bb, py = pp / 14, px = pp - 14 * py;
    const int r = 18 * bb + py - R0;
    pb[i] = (r << 16) | (r * 18 + px);
  }
  auto load_a = [&](int i, int kh, int kw) {
    const int r = (pb[i] >> 16) + 4 - kh, pix = (pb[i] & 0xffff) + (4 - kh) * 18 + 4 - kw;
    const uint32_t* p = img + pix * X6D_PS + 4 * ((4 * h + lg) ^ x6d_swz(pix, r));
    X9Frag f;
    f.p[0] = *reinterpret_cast<const bf16x8*>(p);
    f.p[1] = *reinterpret_cast<const bf16x8*>(p + X6D_PLANE);
    f.p[2] = *reinterpret_cast<const bf16x8*>(p + 2 * X6D_PLANE);
    return f;
  };
  // the running sums alternate sign tap by tap (x9_neg: the bf16 MFMA's rounding bias cancels over
  // consecutive taps); after tap s they hold (-1)^s times the partial sum
  for (int s = 0; s < ntap; ++s) {  // wave-uniform
    const int tap = tap0 + s, kh = tap / 5, kw = tap - 5 * kh;
    X9Frag wb = x9_split8(wraw[0], wraw[1]);
    if (s & 1) wb = x9_neg(wb);
    if (s + 1 < ntap) load_w(tap + 1);
    X9Frag fa = load_a(0, kh, kw);
#pragma unroll
    for (int i = 0; i < TPB; ++i) {
      X9Frag fn;
      if (i + 1 < TPB) fn = load_a(i + 1, kh, kw);
      // pinned: the next tile's reads issue ahead of this tile's MFMAs (left alone, the scheduler
      // waits on each read right before its MFMAs: the LDS latency was exposed every tile)
      __builtin_amdgcn_sched_barrier(0);
      acc[i] = x9_mma<NPROD>(fa, wb, acc[i]);
      __builtin_amdgcn_sched_barrier(0);
      if (i + 1 < TPB) fa = fn;
      if (s + 1 < ntap) acc[i] = f4neg(acc[i]);
    }
  }
  if ((ntap - 1) & 1) {  // wave-uniform: back to the partial sum's own sign
#pragma unroll
    for (int i = 0; i < TPB; ++i) acc[i] = f4neg(acc[i]);
  }
  // the epilogue's conv1 operands (as the native form; loaded after the tap loop, whose registers
  // the accumulators need): (nt, tile) pairs p = wave + 8k
  const int nt = wave & 1;
  constexpr int NP = (2 * TPB + 7) / 8;
  float ea[NP][4];
  int ex[NP][4];
#pragma unroll
  for (int k = 0; k < NP; ++k)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int pp = wave + 8 * k;
      const int P = 16 * (T0 + (pp >> 1)) + 4 * lg + r;
      const bool ok = pp < 2 * TPB && P < np;
      const int64_t o = (int64_t)min(P, np - 1) * 32 + 16 * nt + lr;
      ea[k][r] = mask_f(a1[o], ok);
      ex[k][r] = idx1[o];
    }
  __syncthreads();  // every wave is done with the planes
#pragma unroll
  for (int it = 0; it < 4; ++it) {  // (complete after the next barrier)
    const int i = t + 512 * it, sl = i >> 10, pix = i & 1023;
    xim[sl * CBF_XIMG + (pix >> 5) * CBF_XS + (pix & 31)] = xv[it];
  }
  // 2. the four K-part partials of each (ci group, tile) in the native form's layout
  f32x4* red = reinterpret_cast<f32x4*>(smf);  // [K part][ci group][TPB][64]
#pragma unroll
  for (int i = 0; i < TPB; ++i) red[((kp * 2 + cg) * TPB + i) * 64 + lane] = acc[i];
  __syncthreads();
  // 3. epilogue (the native form's): mask -> g1, conv1 weight gradient of the routed g1, db1
  float s25[26];
#pragma unroll
  for (int e = 0; e < 26; ++e) s25[e] = 0.f;
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int p = wave + 8 * k;  // wave-uniform; p & 1 == nt
    if (p >= 2 * TPB) break;
    const int i = p >> 1;
    const f32x4 sum = ((red[((0 * 2 + nt) * TPB + i) * 64 + lane] + red[((1 * 2 + nt) * TPB + i) * 64 + lane]) +
                       red[((2 * 2 + nt) * TPB + i) * 64 + lane]) +
                      red[((3 * 2 + nt) * TPB + i) * 64 + lane];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int P = 16 * (T0 + i) + 4 * lg + r;
      if (P < np) {
        const int bb = P / 196, pp = P - 196 * bb, py = pp / 14, px = pp - 14 * py;
        const float gv = ea[k][r] > 0.f ? sum[r] : 0.f;
        const int ix = ex[k][r];
        const float* xs = xim + (bb - b0) * CBF_XIMG + (2 * py + (ix >> 1)) * CBF_XS + 2 * px + (ix & 1);
#pragma unroll
        for (int kh = 0; kh < 5; ++kh)
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) s25[kh * 5 + kw] = fmaf(gv, xs[kh * CBF_XS + kw], s25[kh * 5 + kw]);
        s25[25] += gv;
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 26; ++e) {
    float v = s25[e];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    s25[e] = v;
  }
  if (lg == 0) {
#pragma unroll
    for (int e = 0; e < 26; ++e) pw[(wave * 26 + e) * 16 + lr] = s25[e];
  }
  __syncthreads();
  for (int qq = t; qq < CP_F32; qq += 512) {
    const int e = qq >> 5, c = qq & 31, hh = c >> 4, l = c & 15;
    const float v = (pw[((hh + 0) * 26 + e) * 16 + l] + pw[((hh + 2) * 26 + e) * 16 + l]) +
                    (pw[((hh + 4) * 26 + e) * 16 + l] + pw[((hh + 6) * 26 + e) * 16 + l]);
    cpart[(int64_t)bid * CP_F32 + qq] = v;
  }
}

// ------------------------------------------------------------------------------------------ //
// wgrad role on split-bf16 products: dW2[kh][kw][ci][co half] over an image group, as the native role
// (M = 32 co, N = 32 ci per kw: five 32x32 tiles, K = pixels), on v_mfma_f32_32x32x16_bf16 with the
// NPROD part products. Both operands are K-strided in their natural [pixel][channel] layouts, so they
// are staged as bf16 planes of those layouts and read TRANSPOSED: ds_read_b64_tr_b16 delivers, per
// 16-lane group, column i of four rows to lane i (bench_native/tr16_probe.hip), the rows' addresses
// coming from the lanes -- so the kw shift of the a1 operand and the 14-pixel row wrap are just row
// addresses, no copies. Per image: a1 padded rows kh .. kh + 13 ([252 pixels][32 ci] per plane) and
// the dY2 channel half ([196 pixels + 16 zero rows][32 co]); 13 k chunks of 16 pixels, the 91 of a
// 7-image group dealt round-robin over the 8 waves (chunk n * 13 + kc to wave (n * 13 + kc) % 8),
// the next image's loads in registers during the current one. Sign-alternating accumulation as in
// the dgrad role. The partial exchange and the slab writes are the native role's.
constexpr int X6W_A1PL = 252 * 16;                      // dwords per a1 plane
constexpr int X6W_DYPL = 212 * 16;                      // dwords per dY2 plane (16 zero rows)
constexpr int X6W_LDS = (3 * X6W_A1PL + 3 * X6W_DYPL) * 4;   // 89,088 B
static_assert(4 * 5 * 4 * 64 * 16 <= X6W_LDS, "split wgrad exchange fits the planes");
typedef short x6w_v4s __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 x6w_tr8(const uint32_t* row0, const uint32_t* row1) {
  // two transposed reads: elements 0..3 from the first four rows, 4..7 from the next four
  const x6w_v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) x6w_v4s*)row0);
  const x6w_v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) x6w_v4s*)row1);
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, c);
}

template <int NPROD>
__device__ __forceinline__ f32x16 x6w_mma(const X9Frag& a, const X9Frag& b, f32x16 c) {
  auto m = [](const bf16x8& x, const bf16x8& y, f32x16 acc) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, y, acc, 0, 0, 0);
  };
  if constexpr (NPROD == 9) {
    c = m(a.p[2], b.p[2], c);
    c = m(a.p[2], b.p[1], c);
    c = m(a.p[1], b.p[2], c);
  }
  c = m(a.p[2], b.p[0], c);
  c = m(a.p[0], b.p[2], c);
  c = m(a.p[1], b.p[1], c);
  c = m(a.p[1], b.p[0], c);
  c = m(a.p[0], b.p[1], c);
  return m(a.p[0], b.p[0], c);
}

template <int NPROD>
__device__ __forceinline__ void f32x_conv2_wgrad_block(int bid, const float* __restrict__ dY2,
                                                       const float* __restrict__ a1, float* __restrict__ slab, int B,
                                                       int ig, float* smf) {
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int grp = bid / 10, rem = bid - 10 * grp, kh = rem >> 1, ch = rem & 1;
  const int img0 = ig * grp, nimg = min(ig, B - img0);
  uint32_t* a1p = reinterpret_cast<uint32_t*>(smf);
  uint32_t* dyp = a1p + 3 * X6W_A1PL;
  // staging chunks (as the native role): i < 2016 an a1 chunk of the padded rows kh..kh+13, the rest
  // dY2 chunks; the LDS dword offset of each chunk's 4 channels within a plane
  int loff[7], soff[7];
  bool lin[7], la1[7];
#pragma unroll
  for (int it = 0; it < 7; ++it) {
    const int i = t + 512 * it;
    if (i < 2016) {
      const int ly = i / 144, r2 = i - 144 * ly, c = r2 >> 3, q4 = r2 & 7;
      const int y = ly + kh - 2, xx = c - 2;
      const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
      loff[it] = ((in ? y : 0) * 14 + (in ? xx : 0)) * 32 + 4 * q4;
      lin[it] = in;
      la1[it] = true;
      soff[it] = (ly * 18 + c) * 16 + 2 * q4;
    } else {
      const int j = i - 2016, q = j >> 3, q4 = j & 7;
      loff[it] = q * 64 + 32 * ch + 4 * q4;
      lin[it] = i < 3584;
      la1[it] = false;
      soff[it] = 3 * X6W_A1PL + q * 16 + 2 * q4;
    }
  }
  auto load_img = [&](int b, float4 (&v)[7]) {
    const float* pa = a1 + (int64_t)b * 6272;
    const float* pd = dY2 + (int64_t)b * 12544;
#pragma unroll
    for (int it = 0; it < 7; ++it)
      v[it] = mask_f4(*reinterpret_cast<const float4*>((la1[it] ? pa : pd) + (lin[it] ? loff[it] : 0)), lin[it]);
  };
  auto store_img = [&](const float4 (&v)[7]) {
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      if (t + 512 * it < 3584) {
        uint2 h, m, l;
        x9_split4(v[it], h, m, l);
        const int pl = la1[it] ? X6W_A1PL : X6W_DYPL;
        *reinterpret_cast<uint2*>(a1p + soff[it]) = h;
        *reinterpret_cast<uint2*>(a1p + soff[it] + pl) = m;
        *reinterpret_cast<uint2*>(a1p + soff[it] + 2 * pl) = l;
      }
    }
  };
  // the dY2 planes' 16 padding rows (pixels 196..211) are zero for the whole block
  for (int i = t; i < 3 * 16 * 16; i += 512) dyp[(i / 256) * X6W_DYPL + 196 * 16 + (i & 255)] = 0u;
  f32x16 acc[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[k][r] = 0.f;
  float4 v[7];
  load_img(img0, v);
  store_img(v);
  __syncthreads();
  // per-lane transposed-read geometry: group G (l >> 4) reads rows 8 (G >> 1) + 4 r + qq of the chunk,
  // columns 16 (G & 1) + 4 p .. + 3 (lane 4 qq + p of the group)
  const int G = lane >> 4, ii = lane & 15, qq = ii >> 2, pp = ii & 3;
  const int colw = 8 * (G & 1) + 2 * pp;  // dword offset of the lane's 4 columns within a 64-byte row
  int nch = 0;                             // this wave's chunks so far (sign alternation)
  for (int n = 0; n < nimg; ++n) {
    if (n + 1 < nimg) load_img(img0 + n + 1, v);
    const int k0 = (((wave - 13 * n) % 8) + 8) % 8;
    for (int kc = k0; kc < 13; kc += 8) {  // wave-uniform
      const bool neg = nch & 1;
      // rows (pixels) of this lane's two transposed reads
      const int qa = 16 * kc + 8 * (G >> 1) + qq, qb = qa + 4;
      X9Frag fa;
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        fa.p[pl] = x6w_tr8(dyp + pl * X6W_DYPL + qa * 16 + colw, dyp + pl * X6W_DYPL + qb * 16 + colw);
      if (neg) fa = x9_neg(fa);
      const int ca = min(qa, 195), cb = min(qb, 195);  // (padding pixels: dY2 is zero there)
      const int pa = (ca / 14) * 18 + ca % 14, pb = (cb / 14) * 18 + cb % 14;
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        X9Frag fb;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          fb.p[pl] = x6w_tr8(a1p + pl * X6W_A1PL + (pa + kw) * 16 + colw, a1p + pl * X6W_A1PL + (pb + kw) * 16 + colw);
        acc[kw] = x6w_mma<NPROD>(fa, fb, acc[kw]);
      }
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) acc[kw] = -acc[kw];
      ++nch;
    }
    if (n + 1 < nimg) {
      __syncthreads();  // every wave is done with this image's planes
      store_img(v);
      __syncthreads();
    }
  }
  if (nch & 1) {  // one flip per chunk: after an odd number the sums carry a minus sign
#pragma unroll
    for (int kw = 0; kw < 5; ++kw) acc[kw] = -acc[kw];
  }
  __syncthreads();  // the planes are dead: the exchange reuses them
  // partial exchange and slab writes: the native role's
  float4* xr = reinterpret_cast<float4*>(smf);
  if (wave >= 4) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        xr[(((wave - 4) * 5 + kw) * 4 + g) * 64 + lane] =
            make_float4(acc[kw][4 * g], acc[kw][4 * g + 1], acc[kw][4 * g + 2], acc[kw][4 * g + 3]);
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 o = xr[((wave * 5 + kw) * 4 + g) * 64 + lane];
        acc[kw][4 * g] += o.x;
        acc[kw][4 * g + 1] += o.y;
        acc[kw][4 * g + 2] += o.z;
        acc[kw][4 * g + 3] += o.w;
      }
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int kw = 0; kw < 5; ++kw)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        xr[((wave * 5 + kw) * 4 + g) * 64 + lane] =
            make_float4(acc[kw][4 * g], acc[kw][4 * g + 1], acc[kw][4 * g + 2], acc[kw][4 * g + 3]);
  }
  __syncthreads();
  for (int it = t; it < 1280; it += 512) {
    const int kw = it >> 8, g = (it >> 6) & 3, ln = it & 63;
    const float4 a = xr[((0 * 5 + kw) * 4 + g) * 64 + ln], b = xr[((1 * 5 + kw) * 4 + g) * 64 + ln];
    const float4 c = xr[((2 * 5 + kw) * 4 + g) * 64 + ln], d = xr[((3 * 5 + kw) * 4 + g) * 64 + ln];
    const float4 s = make_float4((a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                                 (a.w + b.w) + (c.w + d.w));
    const int tap = kh * 5 + kw, ci = ln & 31, co = 32 * ch + 8 * g + 4 * (ln >> 5);
    *reinterpret_cast<float4*>(slab + (int64_t)grp * 51200 + (tap * 32 + ci) * 64 + co) = s;
  }
}

// conv2_bwd with both roles on split-bf16 products
template <int TPB, int NPROD>
__global__ void __launch_bounds__(512) f32x_conv2_bwd_kernel(
    const float* __restrict__ dY2, const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ idx1, const float* __restrict__ x, const int* __restrict__ rows, int n_pool,
    const int64_t* __restrict__ state, float* __restrict__ cpart, float* __restrict__ slab, int B, int n_dg,
    int n_wg, int ig) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int bid = blockIdx.x;
  if (bid < n_dg) {
    f32x_conv2_dgrad_block<TPB, NPROD>(bid, dY2, w2, a1, idx1, x, rows, n_pool, state, cpart, B, smf);
    return;
  }
  f32x_conv2_wgrad_block<NPROD>(xcd_contiguous(bid, n_dg, n_dg + n_wg), dY2, a1, slab, B, ig, smf);
}

template <int TPB, int NPASS = 1, bool FRAG = false>
__global__ void __launch_bounds__(512) f32_conv2_bwd_kernel(
    const float* __restrict__ dY2, const float* __restrict__ w2, const float* __restrict__ a1,
    const uint8_t* __restrict__ idx1, const float* __restrict__ x, const int* __restrict__ rows, int n_pool,
    const int64_t* __restrict__ state, float* __restrict__ cpart, float* __restrict__ slab, int B, int n_dg,
    int n_wg, int ig, const float* __restrict__ w2f, const float* __restrict__ zeros) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int bid = blockIdx.x;
  c2b_stamp(0);
  if (bid < n_dg) {
    f32_conv2_dgrad_block<TPB, NPASS, FRAG>(bid, dY2, w2, a1, idx1, x, rows, n_pool, state, cpart, B, smf, w2f);
    return;
  }
  // XCD-contiguous order of the wgrad blocks
  f32_conv2_wgrad_block(xcd_contiguous(bid, n_dg, n_dg + n_wg), dY2, a1, slab, B, ig, smf, zeros);
}

// ------------------------------------------------------------------------------------------ //
// f32_conv_reduce: a latency-bound gather of partial sums (the slabs were just written by
// conv2_bwd on every XCD, so most reads miss this XCD's L2), written for memory-level
// parallelism: each thread keeps 8 independent loads in flight and the partial sums meet in LDS.
//   blocks [0, 200):   dW2, 64 float4 per block x 4 slab quarters (sum over the G slabs)
//   blocks [200, 213): dW1 | db1, 16 float4 columns (64 of the 832) x 16 row parts of cpart
//   block  213:        db2, 16 float4 columns x 16 row parts of db2p
//   blocks [214, 214 + n_fc): Adam of the small fc parameters [fc_lo, fc_hi)
// With the optimizer fused (world size 1: the gradients are final here) every element is updated
// by the thread that finishes its gradient and block 0 advances the forward step counter
// (adam_step's bump): one launch for the gradient reduction and the whole optimizer except
// dense/kernel (whose update runs in f32_fc1_bwd from the gradient in registers).
// Fixed summation order (deterministic, no atomics).
// ------------------------------------------------------------------------------------------ //
struct F32SmallAdam {
  F32Adam a;               // p, g, m, v: the FLAT buffers (a.n4 unused); a.nblk = 0: no optimizer
  int o_w1 = 0, o_b1 = 0, o_w2 = 0, o_b2 = 0;   // element offsets of the conv segments
  int fc_lo = 0, fc_hi = 0;                     // the small fc range (multiple-of-4 bounds)
};
constexpr int CR_W2 = 200, CR_CP = 13, CR_DB = 1, CR_FC0 = CR_W2 + CR_CP + CR_DB;

// sum of rows r0, r0 + step, ... (< n) of a float4 column, 8 loads in flight per round
__device__ __forceinline__ float4 strided_sum8(const float4* __restrict__ p, int64_t stride4, int r0, int step, int n) {
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = r0; r < n; r += 8 * step) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int rr = r + u * step;
      v[u] = rr < n ? p[(int64_t)rr * stride4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = f4add(acc, v[u]);
  }
  return acc;
}

__device__ __forceinline__ void adam_flat4(const F32SmallAdam& sa, int64_t o, float4 g, const AdamCoef& c) {
  float4 pp = *reinterpret_cast<const float4*>(sa.a.p + o);
  float4 mm = *reinterpret_cast<const float4*>(sa.a.m + o);
  float4 vv = *reinterpret_cast<const float4*>(sa.a.v + o);
  adam4_f32(pp, mm, vv, g, c);
  *reinterpret_cast<float4*>(sa.a.p + o) = pp;
  *reinterpret_cast<float4*>(sa.a.m + o) = mm;
  *reinterpret_cast<float4*>(sa.a.v + o) = vv;
}

__global__ void __launch_bounds__(256) f32_conv_reduce_kernel(const float* __restrict__ slab, int G,
                                                              const float* __restrict__ cpart, int ncp,
                                                              const float* __restrict__ db2p, int ndb,
                                                              float* __restrict__ gW2, float* __restrict__ gW1,
                                                              float* __restrict__ gb1, float* __restrict__ gb2,
                                                              F32SmallAdam sa, int n_fc) {
  __shared__ float4 red[256];
  const int bid = blockIdx.x, t = threadIdx.x;
  const bool opt = sa.a.nblk > 0;
  AdamCoef c{};
  if (opt) {
    c = f32_adam_coef(sa.a);
    if (bid == 0 && t == 0) const_cast<int64_t*>(sa.a.state)[ST_FWD] += 1;
  }
  if (bid >= CR_FC0) {  // small fc parameters: gradients already final (fc1_bwd)
    const int64_t i = sa.fc_lo / 4 + (int64_t)(bid - CR_FC0) * 256 + t;
    if (opt && i < sa.fc_hi / 4) {
      const float4 gg = reinterpret_cast<const float4*>(sa.a.g)[i];
      adam_flat4(sa, 4 * i, gg, c);
    }
    return;
  }
  const int col = t & 63, part = t >> 6;  // dW2 blocks: 64 float4 x 4 slab quarters
  const int col16 = t & 15, part16 = t >> 4;  // cpart / db2 blocks: 16 float4 columns x 16 row parts
  // this thread's partial-sum rows: one round of 8 loads covers the dW2 slabs and the cpart rows
  // (G <= 32, dgrad blocks <= 128); the db2 rows take the looping strided_sum8
  const float4* sbase;
  int64_t sstride;
  int sr0, sstep, sn;
  if (bid < CR_W2) {
    sbase = reinterpret_cast<const float4*>(slab) + (int64_t)bid * 64 + col;
    sstride = 51200 / 4, sr0 = part, sstep = 4, sn = G;
  } else if (bid < CR_W2 + CR_CP) {
    sbase = reinterpret_cast<const float4*>(cpart) + (bid - CR_W2) * 16 + col16;
    sstride = CP_F32 / 4, sr0 = part16, sstep = 16, sn = ncp;
  } else {
    sbase = reinterpret_cast<const float4*>(db2p) + col16;
    sstride = 16, sr0 = part16, sstep = 16, sn = ndb;
  }
  const bool one = sn <= 8 * sstep;  // block-uniform
  float4 sl[8];
  if (one) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int rr = sr0 + u * sstep;
      sl[u] = rr < sn ? sbase[(int64_t)rr * sstride] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // the Adam operands (p, m, v) of the elements this thread will update, issued right behind the
  // partial-sum loads (pinned) so the two latencies overlap; the sums then wait for their own loads
  // alone (as a loop, the sums' loads had waited for the Adam operands to arrive first)
  float4 pp{}, mm{}, vv{};
  int64_t ao = -1;
  if (opt) {
    if (bid < CR_W2) {
      if (t < 64) ao = sa.o_w2 + 4 * ((int64_t)bid * 64 + t);
    } else if (t < 16) {
      if (bid < CR_W2 + CR_CP) {
        const int q0 = ((bid - CR_W2) * 16 + t) * 4;
        ao = q0 < 800 ? sa.o_w1 + q0 : sa.o_b1 + (q0 - 800);
      } else {
        ao = sa.o_b2 + 4 * t;
      }
    }
    if (ao >= 0 && bid < CR_W2) {  // the W2 segment is float4-aligned (checked on the host)
      pp = *reinterpret_cast<const float4*>(sa.a.p + ao);
      mm = *reinterpret_cast<const float4*>(sa.a.m + ao);
      vv = *reinterpret_cast<const float4*>(sa.a.v + ao);
    } else if (ao >= 0) {  // W1 / b1 / b2: no alignment guarantee, scalar loads
      const float* P = sa.a.p + ao;
      const float* M = sa.a.m + ao;
      const float* V = sa.a.v + ao;
      pp = make_float4(P[0], P[1], P[2], P[3]);
      mm = make_float4(M[0], M[1], M[2], M[3]);
      vv = make_float4(V[0], V[1], V[2], V[3]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  float4 s;
  if (one) {  // the same order of additions as strided_sum8's single round
    s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 8; ++u) s = f4add(s, sl[u]);
  } else {
    s = strided_sum8(sbase, sstride, sr0, sstep, sn);
  }
  red[t] = s;
  __syncthreads();
  if (bid < CR_W2) {
    if (t < 64) {
      const float4 g = f4add(f4add(red[t], red[64 + t]), f4add(red[128 + t], red[192 + t]));
      const int64_t i = (int64_t)bid * 64 + t;
      reinterpret_cast<float4*>(gW2)[i] = g;
      if (opt) {
        adam4_f32(pp, mm, vv, g, c);
        *reinterpret_cast<float4*>(sa.a.p + ao) = pp;
        *reinterpret_cast<float4*>(sa.a.m + ao) = mm;
        *reinterpret_cast<float4*>(sa.a.v + ao) = vv;
      }
    }
    return;
  }
  if (t < 16) {
    float4 g = red[t];
#pragma unroll
    for (int q = 1; q < 16; ++q) g = f4add(g, red[16 * q + t]);
    const float ge[4] = {g.x, g.y, g.z, g.w};
    if (bid < CR_W2 + CR_CP) {
      const int q0 = ((bid - CR_W2) * 16 + t) * 4;  // 0..831, a float4 never straddles 800
      if (q0 < 800) {
        *reinterpret_cast<float4*>(gW1 + q0) = g;
      } else {
        *reinterpret_cast<float4*>(gb1 + (q0 - 800)) = g;
      }
    } else {
      *reinterpret_cast<float4*>(gb2 + 4 * t) = g;
    }
    if (opt) {  // the prefetched operands (ao: this block's W1/b1 or b2 elements)
      float* pe = &pp.x;
      float* me = &mm.x;
      float* ve = &vv.x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        adam1(pe[e], me[e], ve[e], ge[e], c);
        sa.a.p[ao + e] = pe[e];
        sa.a.m[ao + e] = me[e];
        sa.a.v[ao + e] = ve[e];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ //
// host wrappers
// ------------------------------------------------------------------------------------------ //
static void chk_f32(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous() && t.numel() == numel, what,
              ": expected a contiguous fp32 device tensor of ", numel, " elements");
}

// Study instrument: a device buffer of [n_blocks][16] shader-clock stamps that f32_conv2_bwd fills
// from now on (n_blocks = 0: off). Returns the buffer (int64).
void f32_fwd_stamps_set(unsigned long long* p);  // f32_fwd.hip

at::Tensor f32_stamps_enable(int64_t n_blocks, int64_t kernel) {
  static at::Tensor buf[3];
  TORCH_CHECK(kernel >= 0 && kernel <= 2, "f32_stamps_enable: kernel 0 = conv2_bwd, 1 = conv2_fwd, 2 = fc1_bwd");
  unsigned long long* p = nullptr;
  if (n_blocks > 0) {
    buf[kernel] = at::zeros({n_blocks * 16}, at::TensorOptions().dtype(at::kLong).device(at::kCUDA));
    p = reinterpret_cast<unsigned long long*>(buf[kernel].data_ptr<int64_t>());
  } else {
    buf[kernel] = at::Tensor();
  }
  if (kernel == 0) {
    TORCH_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_c2b_stamps), &p, sizeof(p)) == hipSuccess, "f32_stamps_enable");
  } else if (kernel == 2) {
    TORCH_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_f1r_stamps), &p, sizeof(p)) == hipSuccess, "f32_stamps_enable");
  } else {
    f32_fwd_stamps_set(p);
  }
  return n_blocks > 0 ? buf[kernel] : at::zeros({0}, at::TensorOptions().dtype(at::kLong));
}

int64_t f32_db2_rows(int64_t B) { return 49 * ((B + 15) / 16); }
static int conv2b_tpb(int B) {
  const int nt = (196 * B + 15) / 16;
  return std::min(7, std::max(1, (nt + 255) / 256));
}
// One-round form (wherever it applies): dgrad blocks of twice the tiles
// in two tap-loop passes and wgrad blocks of twice the images, so both roles fit the CUs in one
// round (B = 100: 123 + 130 = 253 blocks) instead of two (245 + 250): W2 is loaded once per two
// passes, the halo rows are staged once for twice the pixels, and no block starts behind another.
static bool conv2b_one_round(int B) { return 2 * conv2b_tpb(B) <= 10; }
static int conv2b_block_tiles(int B) { return conv2b_one_round(B) ? 2 * conv2b_tpb(B) : conv2b_tpb(B); }
static int conv2b_images(int B) { return conv2b_one_round(B) ? CBF_IG2 : CBF_IG; }
// The split-bf16 roles (f32x_conv2_bwd_kernel): dgrad blocks of up to 10 tiles, the wgrad role the
// CUs they leave (images per group chosen so both roles fit one round of blocks). Measured at B = 100
// (profiles/r06/conv2_bwd_split_balance_r06q2.txt): 10 tiles + 8-image groups (123 + 130 blocks)
// 34.1 us; 12 + 7 (103 + 150) 35.3 us; 11 tiles needs 7-image groups to stay in one round of blocks
// (262 blocks: 54.9 us) or 8 (36.8 us).
static int conv2bx_tiles(int B) {
  const int nt = (196 * B + 15) / 16;
  return std::min(10, std::max(1, (nt + 99) / 100));
}
static int conv2bx_images(int B) {
  const int nt = (196 * B + 15) / 16, tpb = conv2bx_tiles(B), n_dg = (nt + tpb - 1) / tpb;
  const int free = std::max(10, device_cu_count() - n_dg);
  return std::min(B, std::max(1, (10 * B + free - 1) / free));
}
int64_t f32_wgrad_groups(int64_t B, int64_t products) {
  const int ig = products ? conv2bx_images((int)B) : conv2b_images((int)B);
  return (B + ig - 1) / ig;
}
int64_t f32_dgrad_blocks(int64_t B, int64_t products) {
  const int tpb = products ? conv2bx_tiles((int)B) : conv2b_block_tiles((int)B), nt = (196 * (int)B + 15) / 16;
  return (nt + tpb - 1) / tpb;
}

// F32Adam of the fc1 row kernel (f32_fwd.hip builds the others)
static F32Adam f32_fc1_adam(at::Tensor& w3, const c10::optional<at::Tensor>& m3, const c10::optional<at::Tensor>& v3,
                            const c10::optional<at::Tensor>& state, double lr, double b1, double b2, double eps,
                            double gscale, int64_t rule) {
  F32Adam a;
  if (!(m3.has_value() && m3->defined())) return a;
  TORCH_CHECK(v3.has_value() && v3->defined() && state.has_value() && state->defined(),
              "f32_fc1_bwd: the fused dense/kernel Adam needs m3, v3 and the step state");
  for (const at::Tensor* t : {&*m3, &*v3})
    TORCH_CHECK(t->is_cuda() && t->dtype() == at::kFloat && t->is_contiguous() && t->numel() == 3136 * 1024 &&
                    ((uintptr_t)t->data_ptr() & 15) == 0,
                "f32_fc1_bwd: Adam slots must be 16-byte aligned contiguous fp32 [3136 x 1024]");
  TORCH_CHECK(((uintptr_t)w3.data_ptr() & 15) == 0, "f32_fc1_bwd: w3 must be 16-byte aligned");
  a.p = w3.data_ptr<float>();
  a.m = m3->data_ptr<float>();
  a.v = v3->data_ptr<float>();
  a.n4 = 3136 * 1024 / 4;
  a.state = state->data_ptr<int64_t>();
  a.lr = (float)lr;
  a.b1 = (float)b1;
  a.b2 = (float)b2;
  a.eps = (float)eps;
  a.gscale = (float)gscale;
  a.rule = (int)rule;
  a.nblk = 1;
  return a;
}

void f32_fc1_bwd(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& idx2, const at::Tensor& h,
                 const at::Tensor& dlog, at::Tensor& w3, at::Tensor& dY2, at::Tensor& db2p, at::Tensor& gW3,
                 at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, const c10::optional<at::Tensor>& m3,
                 const c10::optional<at::Tensor>& v3, const c10::optional<at::Tensor>& state, double lr, double beta1,
                 double beta2, double eps, double grad_scale, int64_t rule, bool store_w3,
                 const c10::optional<at::Tensor>& px, const c10::optional<at::Tensor>& plabels,
                 const c10::optional<at::Tensor>& prows, const c10::optional<at::Tensor>& pstate,
                 const c10::optional<at::Tensor>& xpre, const c10::optional<at::Tensor>& ypre) {
  const int B = dz.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_fc1_bwd: batch 1..128");
  chk_f32(dz, (int64_t)B * 1024, "f32_fc1_bwd: dz");
  chk_f32(a2, (int64_t)B * 3136, "f32_fc1_bwd: a2");
  TORCH_CHECK(idx2.dtype() == at::kByte && idx2.numel() == (int64_t)B * 3136 && idx2.is_contiguous(), "f32_fc1_bwd: idx2");
  chk_f32(h, (int64_t)B * 1024, "f32_fc1_bwd: h");
  chk_f32(dlog, (int64_t)B * 10, "f32_fc1_bwd: dlog");
  chk_f32(w3, 3136 * 1024, "f32_fc1_bwd: w3");
  chk_f32(dY2, (int64_t)B * 196 * 64, "f32_fc1_bwd: dY2");
  chk_f32(db2p, f32_db2_rows(B) * 64, "f32_fc1_bwd: db2 partial rows");
  chk_f32(gW3, 3136 * 1024, "f32_fc1_bwd: gW3");
  chk_f32(gb3, 1024, "f32_fc1_bwd: gb3");
  chk_f32(gW4, 10240, "f32_fc1_bwd: gW4");
  chk_f32(gb4, 10, "f32_fc1_bwd: gb4");
  const F32Adam ad = f32_fc1_adam(w3, m3, v3, state, lr, beta1, beta2, eps, grad_scale, rule);
  const bool adam = ad.nblk > 0;
  F32Prefetch pf;
  if (ypre.has_value() && ypre->defined()) {
    TORCH_CHECK(px.has_value() && px->defined() && plabels.has_value() && plabels->defined() && prows.has_value() &&
                    prows->defined() && pstate.has_value() && pstate->defined() && xpre.has_value() && xpre->defined(),
                "f32_fc1_bwd: the next batch's gather needs px, plabels, prows, pstate, xpre and ypre");
    const int n_pool = px->size(0);
    TORCH_CHECK(px->is_cuda() && px->dtype() == at::kFloat && px->is_contiguous() && px->dim() == 2 &&
                    px->size(1) == 784, "f32_fc1_bwd: px [n_pool][784]");
    TORCH_CHECK(plabels->dtype() == at::kLong && plabels->is_contiguous() && plabels->numel() == n_pool,
                "f32_fc1_bwd: plabels int64 [n_pool]");
    TORCH_CHECK(prows->dtype() == at::kInt && prows->is_contiguous() && prows->numel() == n_pool,
                "f32_fc1_bwd: prows int32 [n_pool]");
    TORCH_CHECK(pstate->dtype() == at::kLong && pstate->numel() >= ST_WORDS, "f32_fc1_bwd: pstate");
    chk_f32(*xpre, (int64_t)B * 784, "f32_fc1_bwd: xpre [B][784]");
    TORCH_CHECK(ypre->dtype() == at::kInt && ypre->is_contiguous() && ypre->numel() == B, "f32_fc1_bwd: ypre int32 [B]");
    pf.x = px->data_ptr<float>();
    pf.labels = plabels->data_ptr<int64_t>();
    pf.rows = prows->data_ptr<int>();
    pf.state = pstate->data_ptr<int64_t>();
    pf.n_pool = n_pool;
    pf.xpre = xpre->data_ptr<float>();
    pf.ypre = ypre->data_ptr<int>();
  }
  // neither adam nor store_w3: dgrad (+ db3, dW4, db4) only, gW3 untouched (fp32 factor-gather plane)
  const bool dgrad_only = !adam && !store_w3;
  const int G = (B + 15) / 16;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  // Row form: dgrad + dW3 (+ the fused dense/kernel Adam) from one read of W3.
  auto launch = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, F1R_LDS);
    kern<<<F1R_BLOCKS + F1B_SMALL, 512, F1R_LDS, stream>>>(
        dz.data_ptr<float>(), a2.data_ptr<float>(), idx2.data_ptr<uint8_t>(), h.data_ptr<float>(),
        dlog.data_ptr<float>(), w3.data_ptr<float>(), dY2.data_ptr<float>(), db2p.data_ptr<float>(),
        gW3.data_ptr<float>(), gb3.data_ptr<float>(), gW4.data_ptr<float>(), gb4.data_ptr<float>(), B, ad, pf);
  };
  if (dgrad_only) {
    switch (G) {
      case 1: launch(f32_fc1_bwd_rows_kernel<1, false, false>); break;
      case 2: launch(f32_fc1_bwd_rows_kernel<2, false, false>); break;
      case 3: launch(f32_fc1_bwd_rows_kernel<3, false, false>); break;
      case 4: launch(f32_fc1_bwd_rows_kernel<4, false, false>); break;
      case 5: launch(f32_fc1_bwd_rows_kernel<5, false, false>); break;
      case 6: launch(f32_fc1_bwd_rows_kernel<6, false, false>); break;
      case 7: launch(f32_fc1_bwd_rows_kernel<7, false, false>); break;
      default: launch(f32_fc1_bwd_rows_kernel<8, false, false>);
    }
    return;
  }
  // exact wgrad K steps for the headline batch (B = 97..100: 25 instead of 28; bitwise equal to the
  // padded 28, whose extra steps add exact zeros)
  if (G == 7 && (B + 3) / 4 == 25) {
    if (adam && !store_w3) launch(f32_fc1_bwd_rows_kernel<7, true, false, 25>);
    else if (adam) launch(f32_fc1_bwd_rows_kernel<7, true, true, 25>);
    else launch(f32_fc1_bwd_rows_kernel<7, false, true, 25>);
    return;
  }
#define F1R_CASE(GG)                                                       \
  case GG:                                                                 \
    if (adam && store_w3) launch(f32_fc1_bwd_rows_kernel<GG, true, true>); \
    else if (adam) launch(f32_fc1_bwd_rows_kernel<GG, true, false>);       \
    else launch(f32_fc1_bwd_rows_kernel<GG, false, true>);                 \
    break;
  switch (G) {
    F1R_CASE(1)
    F1R_CASE(2)
    F1R_CASE(3)
    F1R_CASE(4)
    F1R_CASE(5)
    F1R_CASE(6)
    F1R_CASE(7)
    default:
      F1R_CASE(8)
  }
#undef F1R_CASE
}

void f32_conv2_bwd(const at::Tensor& dY2, const at::Tensor& w2, const at::Tensor& a1, const at::Tensor& idx1,
                   const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                   at::Tensor& cpart, at::Tensor& slab, const c10::optional<at::Tensor>& w2frag, int64_t products) {
  const int B = a1.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_conv2_bwd: batch 1..128");
  TORCH_CHECK(products == 0 || products == 6 || products == 9, "f32_conv2_bwd: products 0, 6 or 9");
  const float* w2f = nullptr;
  if (w2frag.has_value() && w2frag->defined()) {
    TORCH_CHECK(w2frag->is_cuda() && w2frag->dtype() == at::kFloat && w2frag->is_contiguous() &&
                    w2frag->numel() >= 51200, "f32_conv2_bwd: w2frag (the dgrad fragment copy, 51200 floats)");
    w2f = w2frag->data_ptr<float>();
  }
  chk_f32(dY2, (int64_t)B * 196 * 64, "f32_conv2_bwd: dY2");
  chk_f32(w2, 51200, "f32_conv2_bwd: w2");
  chk_f32(a1, (int64_t)B * 6272, "f32_conv2_bwd: a1");
  TORCH_CHECK(idx1.dtype() == at::kByte && idx1.numel() == (int64_t)B * 6272 && idx1.is_contiguous(), "f32_conv2_bwd: idx1");
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "f32_conv2_bwd: x");
  const bool r1 = conv2b_one_round(B);
  const int n_dg = (int)f32_dgrad_blocks(B, 0), tpb = conv2b_block_tiles(B), ig = conv2b_images(B);
  const int maxr = r1 ? CBF_MAXR2 : CBF_MAXR;
  const int ngrp = (int)f32_wgrad_groups(B, 0);
  if (products == 0) {
    chk_f32(cpart, (int64_t)n_dg * CP_F32, "f32_conv2_bwd: cpart [dgrad blocks][832]");
    chk_f32(slab, (int64_t)ngrp * 51200, "f32_conv2_bwd: slab [groups][51200]");
  }
  const int n_pool = x.size(0);
  const int* rp = nullptr;
  if (rows.has_value() && rows->defined()) {
    TORCH_CHECK(rows->dtype() == at::kInt && rows->numel() == n_pool, "f32_conv2_bwd: rows must be int32 [n_pool]");
    rp = rows->data_ptr<int>();
  } else {
    TORCH_CHECK(n_pool >= B, "f32_conv2_bwd: x has fewer rows than the batch");
  }
  const int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  if (products != 0) {  // split-bf16 dgrad role
    const int n_dg = (int)f32_dgrad_blocks(B, products), tpb = conv2bx_tiles(B), ig = conv2bx_images(B);
    const int ngrp = (int)f32_wgrad_groups(B, products);
    chk_f32(cpart, (int64_t)n_dg * CP_F32, "f32_conv2_bwd: cpart [dgrad blocks][832]");
    chk_f32(slab, (int64_t)ngrp * 51200, "f32_conv2_bwd: slab [groups][51200]");
    for (int blk = 0; blk < n_dg; ++blk) {
      const int P0 = 16 * blk * tpb, P1 = std::min(16 * (blk + 1) * tpb, 196 * B) - 1;
      const int r0 = 18 * (P0 / 196) + (P0 % 196) / 14, r1 = 18 * (P1 / 196) + (P1 % 196) / 14 + 5;
      TORCH_CHECK(r1 - r0 <= X6D_MAXR && P1 / 196 - P0 / 196 <= 1, "f32_conv2_bwd: dgrad tile span exceeds the LDS planes");
    }
    auto stream = c10::hip::getCurrentHIPStream().stream();
    const int lds = std::max(X6D_LDS, X6W_LDS);
    auto launch = [&](auto kern) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      kern<<<n_dg + 10 * ngrp, 512, lds, stream>>>(dY2.data_ptr<float>(), w2.data_ptr<float>(), a1.data_ptr<float>(),
                                                   idx1.data_ptr<uint8_t>(), x.data_ptr<float>(), rp, n_pool, sp,
                                                   cpart.data_ptr<float>(), slab.data_ptr<float>(), B, n_dg, 10 * ngrp,
                                                   ig);
    };
#define C2BX_CASE(T)                                                      \
  case T:                                                                 \
    if (products == 9) launch(f32x_conv2_bwd_kernel<T, 9>);               \
    else launch(f32x_conv2_bwd_kernel<T, 6>);                             \
    break;
    switch (tpb) {
      C2BX_CASE(1)
      C2BX_CASE(2)
      C2BX_CASE(3)
      C2BX_CASE(4)
      C2BX_CASE(5)
      C2BX_CASE(6)
      C2BX_CASE(7)
      C2BX_CASE(8)
      C2BX_CASE(9)
      default:
        C2BX_CASE(10)
    }
#undef C2BX_CASE
    return;
  }
  // host check of the dgrad blocks' row spans (the LDS image) and image count (<= 2)
  for (int blk = 0; blk < n_dg; ++blk) {
    const int P0 = 16 * blk * tpb, P1 = std::min(16 * (blk + 1) * tpb, 196 * B) - 1;
    const int r0 = 18 * (P0 / 196) + (P0 % 196) / 14, r1 = 18 * (P1 / 196) + (P1 % 196) / 14 + 5;
    TORCH_CHECK(r1 - r0 <= maxr && P1 / 196 - P0 / 196 <= 1, "f32_conv2_bwd: dgrad tile span exceeds the LDS image");
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const int lds = r1 ? CBF_LDS2 : CBF_LDS;
  const int grid = n_dg + 10 * ngrp;
  // the wgrad role's next image by LDS-DMA (padding chunks from a zero line); without the zero line
  // the register-staged form
  const float* zl = f32_zero_line(stream);
  auto launch = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kern<<<grid, 512, lds, stream>>>(dY2.data_ptr<float>(), w2.data_ptr<float>(), a1.data_ptr<float>(),
                                     idx1.data_ptr<uint8_t>(), x.data_ptr<float>(), rp, n_pool, sp,
                                     cpart.data_ptr<float>(), slab.data_ptr<float>(), B, n_dg, 10 * ngrp, ig, w2f, zl);
  };
  if (r1) {  // one-round form: 2, 4, ..., 10 tiles in two passes
#define C2B_R1(T)                                                       \
  case T:                                                               \
    if (w2f) launch(f32_conv2_bwd_kernel<T, 2, true>);                  \
    else launch(f32_conv2_bwd_kernel<T, 2>);                            \
    break;
    switch (tpb) {
      C2B_R1(2)
      C2B_R1(4)
      C2B_R1(6)
      C2B_R1(8)
      default:
        C2B_R1(10)
    }
#undef C2B_R1
    return;
  }
#define C2B_CASE(T)                               \
  case T:                                         \
    launch(f32_conv2_bwd_kernel<T>);              \
    break;
  switch (tpb) {
    C2B_CASE(1)
    C2B_CASE(2)
    C2B_CASE(3)
    C2B_CASE(4)
    C2B_CASE(5)
    C2B_CASE(6)
    default:
      C2B_CASE(7)
  }
#undef C2B_CASE
}

void f32_conv_reduce(const at::Tensor& slab, const at::Tensor& cpart, const at::Tensor& db2p, at::Tensor& gW2,
                     at::Tensor& gW1, at::Tensor& gb1, at::Tensor& gb2, const c10::optional<at::Tensor>& params,
                     const c10::optional<at::Tensor>& grads, const c10::optional<at::Tensor>& m,
                     const c10::optional<at::Tensor>& v, const c10::optional<at::Tensor>& state, int64_t o_w1,
                     int64_t o_b1, int64_t o_w2, int64_t o_b2, int64_t fc_lo, int64_t fc_hi, double lr, double b1,
                     double b2, double eps, double grad_scale, int64_t rule) {
  TORCH_CHECK(slab.dtype() == at::kFloat && slab.numel() % 51200 == 0 && slab.numel() > 0, "f32_conv_reduce: slab");
  TORCH_CHECK(cpart.dtype() == at::kFloat && cpart.numel() % CP_F32 == 0 && cpart.numel() > 0, "f32_conv_reduce: cpart");
  TORCH_CHECK(db2p.dtype() == at::kFloat && db2p.numel() % 64 == 0 && db2p.numel() > 0, "f32_conv_reduce: db2p");
  chk_f32(gW2, 51200, "f32_conv_reduce: gW2");
  chk_f32(gW1, 800, "f32_conv_reduce: gW1");
  chk_f32(gb1, 32, "f32_conv_reduce: gb1");
  chk_f32(gb2, 64, "f32_conv_reduce: gb2");
  for (const at::Tensor* t : {(const at::Tensor*)&gW2, (const at::Tensor*)&gW1, (const at::Tensor*)&gb1,
                              (const at::Tensor*)&gb2, &slab, &cpart, &db2p})
    TORCH_CHECK(((uintptr_t)t->data_ptr() & 15) == 0, "f32_conv_reduce: operands must be 16-byte aligned");
  F32SmallAdam sa;
  int n_fc = 0;
  if (params.has_value() && params->defined()) {
    TORCH_CHECK(grads.has_value() && m.has_value() && v.has_value() && state.has_value() && state->defined(),
                "f32_conv_reduce: the fused optimizer needs params, grads, m, v and the step state");
    const int64_t n = params->numel();
    for (const at::Tensor* t : {&*params, &*grads, &*m, &*v})
      TORCH_CHECK(t->is_cuda() && t->dtype() == at::kFloat && t->is_contiguous() && t->numel() == n &&
                      ((uintptr_t)t->data_ptr() & 15) == 0,
                  "f32_conv_reduce: flat fp32 buffers of one length expected");
    TORCH_CHECK(o_w2 % 4 == 0 && fc_lo % 4 == 0 && fc_hi % 4 == 0 && 0 <= fc_lo && fc_lo <= fc_hi && fc_hi <= n,
                "f32_conv_reduce: segment offsets");
    TORCH_CHECK(o_w1 + 800 <= n && o_b1 + 32 <= n && o_w2 + 51200 <= n && o_b2 + 64 <= n,
                "f32_conv_reduce: conv segments exceed the flat buffers");
    TORCH_CHECK(gW2.data_ptr<float>() == grads->data_ptr<float>() + o_w2 &&
                    gW1.data_ptr<float>() == grads->data_ptr<float>() + o_w1 &&
                    gb1.data_ptr<float>() == grads->data_ptr<float>() + o_b1 &&
                    gb2.data_ptr<float>() == grads->data_ptr<float>() + o_b2,
                "f32_conv_reduce: the gradient outputs must be the flat gradient buffer at the given offsets");
    sa.a.p = params->data_ptr<float>();
    sa.a.g = grads->data_ptr<float>();
    sa.a.m = m->data_ptr<float>();
    sa.a.v = v->data_ptr<float>();
    sa.a.state = state->data_ptr<int64_t>();
    sa.a.lr = (float)lr;
    sa.a.b1 = (float)b1;
    sa.a.b2 = (float)b2;
    sa.a.eps = (float)eps;
    sa.a.gscale = (float)grad_scale;
    sa.a.rule = (int)rule;
    sa.a.nblk = 1;
    sa.o_w1 = (int)o_w1;
    sa.o_b1 = (int)o_b1;
    sa.o_w2 = (int)o_w2;
    sa.o_b2 = (int)o_b2;
    sa.fc_lo = (int)fc_lo;
    sa.fc_hi = (int)fc_hi;
    n_fc = (int)((fc_hi - fc_lo) / 4 + 255) / 256;
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  f32_conv_reduce_kernel<<<CR_FC0 + n_fc, 256, 0, stream>>>(
      slab.data_ptr<float>(), (int)(slab.numel() / 51200), cpart.data_ptr<float>(), (int)(cpart.numel() / CP_F32),
      db2p.data_ptr<float>(), (int)(db2p.numel() / 64), gW2.data_ptr<float>(), gW1.data_ptr<float>(),
      gb1.data_ptr<float>(), gb2.data_ptr<float>(), sa, n_fc);
}

}  // namespace mihvd
