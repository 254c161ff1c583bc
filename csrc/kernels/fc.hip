// Dense layers of the MNIST CNN (horovod/tensorflow_mnist.py:64-71):
//   dense   3136 -> 1024 + ReLU + dropout(0.5)   (fc1)
//   dense_1 1024 -> 10 + softmax cross-entropy   (fc2 / "head")
//
// Every GEMM here computes the *transposed* product (output features on the MFMA row axis) so a
// lane's four accumulator rows are four consecutive features of one sample: epilogues store 16 B
// per lane instead of 4 B. Operand tiles are staged with all loads in flight at once
// (stage_tile), so each block pays one memory latency.
//
// fc1_fwd : split-K (16 column tiles x 14 K slices = 224 blocks); each block streams a disjoint
//           28 KB slice of W3 and writes an fp32 partial slab — the step is weight-bandwidth bound.
// head    : one block per sample: slab sum + bias + ReLU + counter-based dropout, fc2, softmax
//           cross-entropy and the fc2 backward into dz (K9-K11 of SURVEY.md §2.5, one kernel).
// fc1_wgrad: one launch, four block roles: dW3 straight into the fusion buffer, db3, dW4, db4
//           (+ zeroing of the gradients conv2_bwd accumulates atomically).
// fc1_dgrad: full-K tiles (W3 rows in registers, dz in LDS) with the pooled-ReLU mask and the
//           bf16 cast fused into the epilogue.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"
#include "xgmi_role.h"

MIHVD_OPNS_BEGIN

constexpr int FC1_K = 3136, FC1_N = 1024, FC1_KS = 7, FC1_KSL = FC1_K / FC1_KS;   // 448 = 14 K steps
constexpr int FC1_NT = 32;                                                          // columns per block
constexpr int MAXB = 128;                                                           // batch limit (8 tiles)
constexpr int F1_ASTR = FC1_KSL + 8;   // a2 image rows: 456 elements (912 B)
constexpr int F1_WSTR = FC1_NT + 8;    // W3 image rows: 40 elements (80 B)
constexpr int F1_LDS = (MAXB * F1_ASTR + FC1_KSL * F1_WSTR) * 2;   // 152,576 B
static_assert(F1_LDS <= 163840, "fc1_fwd LDS image exceeds the CU's 160 KiB");

// grid (32, 7): blockIdx.x = 32-column tile, blockIdx.y = K slice (448 = 14 K steps). NW = 4 or 8
// waves: wave w owns the 16 features w % 2 and the sample-tile group w / 2.
// MT = ceil(B/16) sample tiles, a template parameter (no runtime guard around any MFMA: the odd
// half's spare tile recomputes the last real one and is not stored).
template <int MT, int NW = 4>
__global__ void __launch_bounds__(NW * 64) fc1_fwd_kernel(const u16* __restrict__ a2, const u16* __restrict__ w3,
                                                          float* __restrict__ zpart, int B) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  constexpr int Mpad = MT * 16, T = NW * 64;
  constexpr int WN = FC1_NT / 16, MG = NW / WN;     // 16-feature groups, sample-tile groups
  constexpr int MTW = (MT + MG - 1) / MG;           // sample tiles per wave
  u16* Ws = smem;                     // [448][F1_WSTR]    rows = k, n contiguous
  u16* As = smem + FC1_KSL * F1_WSTR; // [Mpad][F1_ASTR]   rows = samples, k contiguous
  const int nt = blockIdx.x, ks = blockIdx.y, t = threadIdx.x;
  const int k0 = ks * FC1_KSL;
  {
    TileLoad<T, (Mpad * FC1_KSL / 8 + T - 1) / T, FC1_KSL / 8> la;
    TileLoad<T, (FC1_KSL * FC1_NT / 8 + T - 1) / T, FC1_NT / 8> lw;
    lw.load(w3 + (int64_t)k0 * FC1_N + nt * FC1_NT, FC1_N, FC1_KSL, FC1_KSL, t);
    la.load(a2 + k0, FC1_K, Mpad, B, t);
    lw.store(Ws, F1_WSTR, FC1_KSL, t);
    la.store(As, F1_ASTR, Mpad, t);
  }
  __syncthreads();
  const int lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4, q = lr >> 2, p = lr & 3;
  const int wn = wave % WN, mt0 = (wave / WN) * MTW;
  f32x4 acc[MTW];
#pragma unroll
  for (int i = 0; i < MTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < FC1_KSL / 32; ++kk) {
    // A = W3^T (rows = features n), read transposed from the [k][n] image.
    const u16* wr = Ws + (kk * 32 + 8 * lg + q) * F1_WSTR + wn * 16 + 4 * p;
    const bf16x8 afr = frag_tr(wr, wr + 4 * F1_WSTR);
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const int mt = min(mt0 + i, MT - 1);
      const bf16x8 bfr = frag_ld128(As + (mt * 16 + lr) * F1_ASTR + kk * 32 + 8 * lg);
      acc[i] = mfma16(afr, bfr, acc[i]);
    }
  }
  float* out = zpart + (int64_t)ks * B * FC1_N;
  const int n = nt * FC1_NT + wn * 16 + 4 * lg;
#pragma unroll
  for (int i = 0; i < MTW; ++i) {
    const int m = (mt0 + i) * 16 + lr;
    if (mt0 + i < MT && m < B)
      *reinterpret_cast<float4*>(out + (int64_t)m * FC1_N + n) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  }
}

// ------------------------------------------------------------------------------------------ //
// head: one block per sample b, 256 threads x 4 features.
// ------------------------------------------------------------------------------------------ //
__global__ void __launch_bounds__(256) head_kernel(
    const float* __restrict__ zpart, const float* __restrict__ b3, const float* __restrict__ w4,
    const float* __restrict__ b4, const int64_t* __restrict__ labels, const int* __restrict__ rows, int n_pool,
    int64_t* __restrict__ state, uint32_t seed, uint32_t thresh24, float keep_scale, float dz_mul, u16* __restrict__ h_out,
    u16* __restrict__ dz_out, float* __restrict__ dlog_out, float* __restrict__ stats, int B, CollRole cr,
    float* __restrict__ stats_acc, const float* __restrict__ ls) {
  __shared__ float red[4][10];
  __shared__ float dl[10];
  // co-launched xGMI collective (xgmi_role.h) on the first cr.nblk blocks
  if ((int)blockIdx.x < cr.nblk) {
    coll_role_run(cr, blockIdx.x);
    return;
  }
  const int b = blockIdx.x - cr.nblk, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t step = state ? state[ST_FWD] : 0;
  const int n0 = t * 4;
  float4 parts[FC1_KS];
#pragma unroll
  for (int s = 0; s < FC1_KS; ++s) parts[s] = *reinterpret_cast<const float4*>(zpart + ((int64_t)s * B + b) * FC1_N + n0);
  float w4r[4][10];  // this thread's 4 rows of W4 = 40 contiguous floats = 10 x 16 B
  {
    float4 wv[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) wv[k] = reinterpret_cast<const float4*>(w4 + n0 * 10)[k];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const float e[4] = {wv[k].x, wv[k].y, wv[k].z, wv[k].w};
#pragma unroll
      for (int u = 0; u < 4; ++u) w4r[(4 * k + u) / 10][(4 * k + u) % 10] = e[u];
    }
  }
  const float4 bb = *reinterpret_cast<const float4*>(b3 + n0);
  // the label (step -> rows[] -> labels[]: dependent loads) is fetched now, so its latency hides
  // under the fc2 partial sums instead of following the first barrier
  int y = 0;
  if (t < 64) {
    int row = b;
    if (rows != nullptr) row = rows[(int)((step * (int64_t)B + b) % n_pool)];
    y = (int)labels[row];
  }
  float z[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
  for (int s = 0; s < FC1_KS; ++s) {
    z[0] += parts[s].x; z[1] += parts[s].y; z[2] += parts[s].z; z[3] += parts[s].w;
  }
  float h[4];
  u16 hb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool keep = thresh24 == 0 || dropout_keep(seed, (uint32_t)step, (uint32_t)(b * FC1_N + n0 + i), thresh24);
    const float v = keep ? fmaxf(z[i], 0.f) * keep_scale : 0.f;
    hb[i] = f2bf(v);
    h[i] = bf2f(hb[i]);  // fc2 consumes exactly the stored (bf16) activation
  }
  *reinterpret_cast<uint2*>(h_out + (int64_t)b * FC1_N + n0) =
      make_uint2((uint32_t)hb[0] | ((uint32_t)hb[1] << 16), (uint32_t)hb[2] | ((uint32_t)hb[3] << 16));
  float part[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) part[c] = h[0] * w4r[0][c] + h[1] * w4r[1][c] + h[2] * w4r[2][c] + h[3] * w4r[3][c];
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    const float s = wave_sum(part[c]);
    if (lane == 0) red[wave][c] = s;
  }
  __syncthreads();
  if (t < 64) {
    // one wave finishes the 10-way softmax; lanes 0..9 own a class each
    const int c = min(lane, 9);
    const float lg = red[0][c] + red[1][c] + red[2][c] + red[3][c] + b4[c];
    const float v = lane < 10 ? lg : -INFINITY;
    const float mx = wave_max(v);
    const float e = lane < 10 ? __expf(lg - mx) : 0.f;
    const float se = wave_sum(e);
    const float lse = mx + __logf(se);
    // argmax (first max) for the accuracy metric
    const unsigned long long ismax = __ballot(lane < 10 && lg == mx);
    const int am = __ffsll((long long)ismax) - 1;
    const float ly = __shfl(lg, y, 64);
    if (lane < 10) {
      const float d = (__expf(lg - lse) - (lane == y ? 1.f : 0.f)) * (1.0f / (float)B);
      dl[lane] = d;
      // ls (the fused fp16 step's device loss scale [S, found]): dlog is stored S-scaled like dz,
      // so every gradient of the step (dW4 / db4 included) carries S and one unscale fits all
      dlog_out[b * 10 + lane] = ls != nullptr ? d * ls[0] : d;
    }
    if (lane == 0) {
      stats[b * 2 + 0] = lse - ly;
      stats[b * 2 + 1] = (am == y) ? 1.f : 0.f;
      if (stats_acc != nullptr) {  // running per-sample sums (this block is the sample's only writer)
        stats_acc[b * 2 + 0] += lse - ly;
        stats_acc[b * 2 + 1] += (am == y) ? 1.f : 0.f;
      }
      if (b == 0 && state != nullptr) state[ST_OPT] += 1;
    }
  }
  __syncthreads();
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) s = fmaf(dl[c], w4r[i][c], s);
    // dz_mul = keep_scale x the loss scale (fp16 build; with ls the scale is read on the device)
    g[i] = h[i] > 0.f ? s * (ls != nullptr ? dz_mul * ls[0] : dz_mul) : 0.f;
  }
  *reinterpret_cast<uint2*>(dz_out + (int64_t)b * FC1_N + n0) = pack4bf(g[0], g[1], g[2], g[3]);
}

// ------------------------------------------------------------------------------------------ //
// fc1_dgrad: g2[b][j] = (a2[b][j] > 0) * sum_n dz[b][n] W3[j][n]     (no split-K, no combine)
//
// Block = 64 features j x 32 samples x the full K = 1024. Both operands are K-contiguous, so each
// wave keeps its 16 rows of W3 (32 KB) in registers straight from global memory — one 32-byte
// load per lane per 64-wide K step, all 32 loads in flight at once — while the block's 32 dz rows
// (64 KB) are staged once in LDS. The K order inside a 64-wide step is permuted identically for
// both operands (lane group lg owns K = 64s + 16lg + [0,16)), which lets a lane load 32 contiguous
// bytes. The four sample groups of a feature tile are mapped to the same XCD (blockIdx & 7), so
// W3 comes from HBM once per XCD L2 and three of its four reads hit.
// ------------------------------------------------------------------------------------------ //
constexpr int DG_ROWS = 32, DG_JT = FC1_K / 64;         // 49 feature tiles
constexpr int DG_DSTR = FC1_N + 8;                      // dz image row stride (2064 B)
constexpr int DG_LDS = DG_ROWS * DG_DSTR * 2;           // 66,048 B

// FT_KP: row length of the transposed factor copies a2T [3136][128] / dzT [1024][128] that the
// dgrad blocks can leave for conv2_bwd's dW3 tail (w3_tail.h): K-contiguous rows make every MFMA
// fragment there one 16-byte load. Columns past the batch are never written (zero-initialised).
constexpr int FT_KP = MAXB;

__device__ __forceinline__ void fc1_dgrad_block(int bx, const u16* __restrict__ dz, const u16* __restrict__ w3,
                                                const u16* __restrict__ a2, u16* __restrict__ g2, int B, int G,
                                                u16* smem, u16* __restrict__ a2T = nullptr,
                                                u16* __restrict__ dzT = nullptr) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  const int xcd = bx & 7, slot = bx >> 3;
  const int mg = slot % G, jt = (slot / G) * 8 + xcd;
  if (jt >= DG_JT) return;
  const int j0 = jt * 64, m0 = mg * DG_ROWS;
  const int rows = min(DG_ROWS, B - m0);
  // Load order matters: vmcnt retires in issue order, so the dz tile (needed first, for the LDS
  // image) is issued before the 32 W3 loads, which then land while the image is written.
  // 1. the block's dz rows (rows past B zero-filled)
  TileLoad<256, DG_ROWS * (FC1_N / 8) / 256, FC1_N / 8> ld;
  ld.load(dz + (int64_t)m0 * FC1_N, FC1_N, DG_ROWS, rows, t);
  // 2. this wave's W3 rows: j = j0 + 16*wave + lr, K chunk [64s + 16lg, +16) for s = 0..15
  uint4 wv[16][2];
  {
    const u16* wr = w3 + (int64_t)(j0 + wave * 16 + lr) * FC1_N + 16 * lg;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      wv[s][0] = *reinterpret_cast<const uint4*>(wr + 64 * s);
      wv[s][1] = *reinterpret_cast<const uint4*>(wr + 64 * s + 8);
    }
  }
  // 3. pooled-ReLU mask for the epilogue rows (a2 > 0), 4 features per lane
  uint2 mk[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = m0 + mt * 16 + lr;
    const uint2 x = *reinterpret_cast<const uint2*>(a2 + (int64_t)min(m, B - 1) * FC1_K + j0 + wave * 16 + 4 * lg);
    const uint32_t keep = m < B ? 0xffffffffu : 0u;
    mk[mt] = make_uint2(x.x & keep, x.y & keep);
  }
  u16* Ds = smem;
  ld.store(Ds, DG_DSTR, DG_ROWS, t);
  __syncthreads();
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const bf16x8 afr = __builtin_bit_cast(bf16x8, wv[s][hh]);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const bf16x8 bfr = frag_ld128(Ds + (mt * 16 + lr) * DG_DSTR + 64 * s + 16 * lg + 8 * hh);
        acc[mt] = mfma16(afr, bfr, acc[mt]);
      }
    }
  }
  // C[row = 4lg + i][col = lr] = feature j0 + 16*wave + 4lg + i, sample m0 + 16mt + lr
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = m0 + mt * 16 + lr;
    if (m < B) {
      const uint2 x = mk[mt];
      const u16 av[4] = {(u16)(x.x & 0xffff), (u16)(x.x >> 16), (u16)(x.y & 0xffff), (u16)(x.y >> 16)};
      float o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = bf2f(av[i]) > 0.f ? acc[mt][i] : 0.f;
      *reinterpret_cast<uint2*>(g2 + (int64_t)m * FC1_K + j0 + wave * 16 + 4 * lg) = pack4bf(o[0], o[1], o[2], o[3]);
    }
  }
  if (a2T != nullptr) {
    // a2T[j][m] for this block's 64 features x 32 samples (zero past B: mk is masked): lanes lr
    // hold 16 consecutive samples, so each store instruction writes 32 contiguous bytes per row.
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = m0 + mt * 16 + lr;
      const uint2 x = mk[mt];
      const u16 av[4] = {(u16)(x.x & 0xffff), (u16)(x.x >> 16), (u16)(x.y & 0xffff), (u16)(x.y >> 16)};
#pragma unroll
      for (int i = 0; i < 4; ++i) a2T[(int64_t)(j0 + wave * 16 + 4 * lg + i) * FT_KP + m] = av[i];
    }
  }
  if (dzT != nullptr && jt < FC1_N / 64) {
    // dzT[n][m] for n in [64 jt, 64 jt + 64), this block's 32 samples, read from the dz image
    // (rows past B are zero-filled): 8 consecutive samples -> one 16-byte store per thread.
    const int n = jt * 64 + (t & 63), mq = t >> 6;
    u16 e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = Ds[(8 * mq + k) * DG_DSTR + n];
    uint4 v;
    v.x = (uint32_t)e[0] | ((uint32_t)e[1] << 16);
    v.y = (uint32_t)e[2] | ((uint32_t)e[3] << 16);
    v.z = (uint32_t)e[4] | ((uint32_t)e[5] << 16);
    v.w = (uint32_t)e[6] | ((uint32_t)e[7] << 16);
    *reinterpret_cast<uint4*>(dzT + (int64_t)n * FT_KP + m0 + 8 * mq) = v;
  }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) fc1_dgrad_kernel(
    const u16* __restrict__ dz, const u16* __restrict__ w3, const u16* __restrict__ a2, u16* __restrict__ g2, int B,
    int G) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  fc1_dgrad_block(blockIdx.x, dz, w3, a2, g2, B, G, smem);
}

// ------------------------------------------------------------------------------------------ //
// fc1_wgrad roles (dispatch order: the 33 small blocks first, then the 784 dW3 tiles):
//   wgrad : 64x64 tile of dW3 = a2^T dz   (K = batch, zero padded)
//   db3 (16 blocks), dW4 (16 blocks), misc: db4
// ------------------------------------------------------------------------------------------ //
constexpr int FB_WGRAD = (FC1_K / 64) * (FC1_N / 64);            // 784
constexpr int FB_DB3 = FC1_N / 64, FB_DW4 = FC1_N / 64, FB_MISC = 1;  // 16 + 16 + 1 blocks
constexpr int FB_TOTAL = FB_WGRAD + FB_DB3 + FB_DW4 + FB_MISC;
constexpr int FB_TSTR = 64 + 8;                                  // 72 elements
constexpr int FB_LDS_WG = 2 * MAXB * FB_TSTR * 2;                // 36,864 B

// ADAM: the dW3 tiles apply the optimizer to W3 in their epilogue (p, m, v, bf16 shadow of the
// dense/kernel segment) straight from the accumulators, so dW3 never round-trips through HBM; the
// gradient is stored too only when write_grad is set (tests). Valid whenever the tile's dW3 is
// already the full data-parallel sum: world size 1, or the all-gathered factors (Kw = size * B).
template <bool ADAM>
__device__ __forceinline__ void fc1_wgrad_block(
    int bx, const u16* __restrict__ dz, const u16* __restrict__ a2, const u16* __restrict__ h,
    const float* __restrict__ dlog, const u16* __restrict__ dzw, const u16* __restrict__ a2w, int Kw,
    float* __restrict__ gW3, float* __restrict__ gb3, float* __restrict__ gW4, float* __restrict__ gb4, int B,
    int tile_base, int n_small, const AdamArgs& ad, int write_grad, int a2s, int a2c0, u16* smem) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  // The small-reduction blocks (n_small = 33, or 0 when they are not launched) come first in
  // dispatch order so they run alongside the dW3 tiles instead of trailing them.
  // dW3 tiles launched: [tile_base, tile_base + gridDim.x - n_small) (a row-slice of dW3 when the
  // optimizer of dense/kernel is sharded across ranks).
  int bid = bx;
  bid = bid < n_small ? FB_WGRAD + bid : tile_base + (bid - n_small);
  if (bid < FB_WGRAD) {
    // dW3^T[n][j] tile = sum_k dzw[k][n] a2w[k][j] over Kw rows (the local batch, or the batch of
    // every rank when the factors were all-gathered) -> stored as gW3[j][n..n+3] (float4 per lane).
    // K streams through LDS in chunks of 128 rows; the next chunk's loads are in flight while the
    // current one is multiplied.
    const int jt = bid >> 4, ntile = bid & 15;
    const int j0 = jt * 64, n0 = ntile * 64;
    u16* Zim = smem;                   // [128][72]  rows k, cols n
    u16* Aim = smem + MAXB * FB_TSTR;  // [128][72]  rows k, cols j
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;  // wave's 32 (n) x 32 (j) sub-tile
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    TileLoad<256, (MAXB * 8 + 255) / 256, 8> lz, la;
    {
      const int rows = min(MAXB, Kw);
      lz.load(dzw + n0, FC1_N, (rows + 31) & ~31, rows, t);
      la.load(a2w + (j0 - a2c0), a2s, (rows + 31) & ~31, rows, t);
    }
    float4 pp[2][2], mm[2][2], vv[2][2];
    for (int kc = 0; kc < Kw; kc += MAXB) {
      const int rows = min(MAXB, Kw - kc), Kpad = (rows + 31) & ~31;
      if (kc > 0) __syncthreads();  // the previous chunk's fragments have been read
      lz.store(Zim, FB_TSTR, Kpad, t);
      la.store(Aim, FB_TSTR, Kpad, t);
      __syncthreads();
      if constexpr (ADAM) {
        // Optimizer operands of this lane's four float4 outputs: issued once the first operand
        // chunk is in LDS (vmcnt retires in order, so issuing them earlier would make the operand
        // wait include them) and in flight during the MFMA loop.
        if (kc == 0) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
              const int64_t o = (int64_t)(j0 + wn + jj * 16 + lr) * FC1_N + n0 + wm + i * 16 + 4 * lg;
              pp[i][jj] = *reinterpret_cast<const float4*>(ad.p + o);
              mm[i][jj] = *reinterpret_cast<const float4*>(ad.m + o);
              vv[i][jj] = *reinterpret_cast<const float4*>(ad.v + o);
            }
        }
      }
      if (kc + MAXB < Kw) {
        const int nrows = min(MAXB, Kw - kc - MAXB);
        lz.load(dzw + (int64_t)(kc + MAXB) * FC1_N + n0, FC1_N, (nrows + 31) & ~31, nrows, t);
        la.load(a2w + (int64_t)(kc + MAXB) * a2s + (j0 - a2c0), a2s, (nrows + 31) & ~31, nrows, t);
      }
      for (int k0 = 0; k0 < Kpad; k0 += 32) {
        bf16x8 af[2], bfv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const u16* zr = Zim + (k0 + 8 * lg + q) * FB_TSTR + wm + i * 16 + 4 * p;
          af[i] = frag_tr(zr, zr + 4 * FB_TSTR);
          const u16* ar = Aim + (k0 + 8 * lg + q) * FB_TSTR + wn + i * 16 + 4 * p;
          bfv[i] = frag_tr(ar, ar + 4 * FB_TSTR);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mfma16(af[i], bfv[jj], acc[i][jj]);
      }
    }
    if constexpr (ADAM) {
      const AdamCoef c = adam_coef((float)ad.state[ST_OPT], ad.lr, ad.b1, ad.b2, ad.eps, ad.gscale, ad.rule);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int64_t o = (int64_t)(j0 + wn + jj * 16 + lr) * FC1_N + n0 + wm + i * 16 + 4 * lg;
          const float4 g = make_float4(acc[i][jj][0], acc[i][jj][1], acc[i][jj][2], acc[i][jj][3]);
          if (write_grad) *reinterpret_cast<float4*>(gW3 + o) = g;
          const uint2 sh = adam4(pp[i][jj], mm[i][jj], vv[i][jj], g, c);
          *reinterpret_cast<float4*>(ad.p + o) = pp[i][jj];
          *reinterpret_cast<float4*>(ad.m + o) = mm[i][jj];
          *reinterpret_cast<float4*>(ad.v + o) = vv[i][jj];
          *reinterpret_cast<uint2*>(ad.shadow + o) = sh;
        }
      return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int n = n0 + wm + i * 16 + 4 * lg;
        const int j = j0 + wn + jj * 16 + lr;
        *reinterpret_cast<float4*>(gW3 + (int64_t)j * FC1_N + n) =
            make_float4(acc[i][jj][0], acc[i][jj][1], acc[i][jj][2], acc[i][jj][3]);
      }
    return;
  }
  bid -= FB_WGRAD;
  // Small reductions over the batch: thread = (feature n in a 64-wide tile, row group rg of 32
  // samples); every row load of a thread is issued at once (masked past B), then a 4-way LDS sum.
  const int nn = t & 63, rg = t >> 6;
  if (bid < FB_DB3) {
    const int n = bid * 64 + nn;
    float v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int b = rg * 32 + i;
      v[i] = mask_f(bf2f(dz[(int64_t)min(b, B - 1) * FC1_N + n]), b < B);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += v[i];
    float* red = reinterpret_cast<float*>(smem);
    red[rg * 64 + nn] = s;
    __syncthreads();
    if (t < 64) gb3[n] = (red[nn] + red[64 + nn]) + (red[128 + nn] + red[192 + nn]);
    return;
  }
  bid -= FB_DB3;
  if (bid < FB_DW4) {
    float* dls = reinterpret_cast<float*>(smem);  // [B][10]
    float* red = dls + MAXB * 10;                  // [4][64][10]
    const int n = bid * 64 + nn;
    float hv[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int b = rg * 32 + i;
      hv[i] = mask_f(bf2f(h[(int64_t)min(b, B - 1) * FC1_N + n]), b < B);
    }
    for (int i = t; i < B * 10; i += 256) dls[i] = dlog[i];
    for (int i = B * 10 + t; i < MAXB * 10; i += 256) dls[i] = 0.f;
    __syncthreads();
    float s[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) s[c] = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i)
#pragma unroll
      for (int c = 0; c < 10; ++c) s[c] = fmaf(hv[i], dls[(rg * 32 + i) * 10 + c], s[c]);
#pragma unroll
    for (int c = 0; c < 10; ++c) red[(rg * 64 + nn) * 10 + c] = s[c];
    __syncthreads();
    for (int i = t; i < 640; i += 256) {
      const int n2 = i / 10, c = i - n2 * 10;
      gW4[(bid * 64 + n2) * 10 + c] = (red[n2 * 10 + c] + red[(64 + n2) * 10 + c]) +
                                      (red[(128 + n2) * 10 + c] + red[(192 + n2) * 10 + c]);
    }
    return;
  }
  // misc: db4 (thread = class c, row group)
  {
    float* red = reinterpret_cast<float*>(smem);
    const int c = t % 10, g = t / 10;  // 25 groups x 10 classes = 250 threads
    float s = 0.f;
    if (g < 25) {
      float v[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int b = g * 6 + i;  // 25 x 6 = 150 >= MAXB rows
        v[i] = mask_f(dlog[min(b, B - 1) * 10 + c], b < B);
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) s += v[i];
    }
    red[t] = s;
    __syncthreads();
    if (t < 10) {
      float tot = 0.f;
      for (int gg = 0; gg < 25; ++gg) tot += red[gg * 10 + t];
      gb4[t] = tot;
    }
  }
}

template <bool ADAM, int MINW = 1>
__global__ void __launch_bounds__(256, MINW) fc1_wgrad_kernel(
    const u16* __restrict__ dz, const u16* __restrict__ a2, const u16* __restrict__ h, const float* __restrict__ dlog,
    const u16* __restrict__ dzw, const u16* __restrict__ a2w, int Kw, float* __restrict__ gW3, float* __restrict__ gb3,
    float* __restrict__ gW4, float* __restrict__ gb4, int B, int tile_base, int n_small, AdamArgs ad, int write_grad,
    int a2s, int a2c0, CollRole cr) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  if ((int)blockIdx.x < cr.nblk) {  // co-launched xGMI collective (xgmi_role.h)
    coll_role_run(cr, blockIdx.x);
    return;
  }
  fc1_wgrad_block<ADAM>((int)blockIdx.x - cr.nblk, dz, a2, h, dlog, dzw, a2w, Kw, gW3, gb3, gW4, gb4, B, tile_base,
                        n_small, ad, write_grad, a2s, a2c0, smem);
}

// dW3 tiles over a long K (the all-gathered factors of N ranks, Kw = N*B) with the K chunks split
// between the G 4-wave groups of a 256*G-thread block (G = 2 or 4): group g streams chunks g, g+G, ...
// through its own LDS images (the next chunk's loads in flight while it multiplies), so a tile's
// chunk chain is 1/G as long as in fc1_wgrad_block. The groups then exchange their partial tiles
// through LDS and each finishes 4/G of the 2x2 sub-tiles: the sum over groups 0, 1, ..., G-1 in that
// order (deterministic), then the store or the Adam epilogue. Only the tile geometry of
// fc1_wgrad_block is reused; results differ from it in the last bits (the K sum is split) but every
// rank and every row slice computes the same values. G = 4 pays where the chunk chain is long (the
// 8-rank factors: 7 chunks -> 2 per group instead of 4).
template <bool ADAM, int G, int NTW = 64>
__device__ __forceinline__ void fc1_dw3_tile_kg(int tile, const u16* __restrict__ dzw, const u16* __restrict__ a2w,
                                                int Kw, float* __restrict__ gW3, const AdamArgs& ad, int write_grad,
                                                int a2s, int a2c0, u16* smem) {
  static_assert(G == 2 || G == 4, "fc1_dw3_tile_kg: 2 or 4 groups");
  static_assert(NTW == 64 || NTW == 32, "fc1_dw3_tile_kg: 64- or 32-feature tiles");
  constexpr int SI = NTW / 32;                 // 16-feature sub-tile rows per wave (2 or 1)
  constexpr int S = SI * 2;                    // sub-tiles (i, jj) per wave
  constexpr int U = S / G > 0 ? S / G : 1;     // sub-tiles finished by each group (groups g*U >= S idle)
  constexpr int NTILES = FC1_N / NTW;          // feature tiles per 64-row tile row
  const int t = threadIdx.x, g = t >> 8, th = t & 255, lane = th & 63, wave = th >> 6, lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  const int jt = tile / NTILES, ntile = tile - jt * NTILES;
  const int j0 = jt * 64, n0 = ntile * NTW;
  u16* Zim = smem + g * (2 * MAXB * FB_TSTR);  // [128][72] rows k, cols n (NTW used)
  u16* Aim = Zim + MAXB * FB_TSTR;             // [128][72] rows k, cols j
  const int wm = (wave >> 1) * (NTW / 2), wn = (wave & 1) * 32;
  const int nch = (Kw + MAXB - 1) / MAXB, nit = (nch + G - 1) / G;
  auto rows_of = [&](int c) { return c < nch ? min(MAXB, Kw - c * MAXB) : 0; };
  f32x4 acc[SI][2];
#pragma unroll
  for (int i = 0; i < SI; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  TileLoad<256, (MAXB * (NTW / 8) + 255) / 256, NTW / 8> lz;
  TileLoad<256, (MAXB * 8 + 255) / 256, 8> la;
  {
    const int rows = rows_of(g);
    if (rows > 0) {
      lz.load(dzw + (int64_t)g * MAXB * FC1_N + n0, FC1_N, (rows + 31) & ~31, rows, th);
      la.load(a2w + (int64_t)g * MAXB * a2s + (j0 - a2c0), a2s, (rows + 31) & ~31, rows, th);
    }
  }
  const bool fin = g * U < S;  // this group finishes sub-tiles
  float4 pp[U], mm[U], vv[U];  // Adam operands of this group's sub-tiles u = g*U + s (i = u >> 1, jj = u & 1)
  for (int it = 0; it < nit; ++it) {
    const int c = G * it + g;
    const int rows = rows_of(c), Kpad = (rows + 31) & ~31;
    if (it > 0) __syncthreads();  // every group read its previous chunk's fragments
    if (rows > 0) {
      lz.store(Zim, FB_TSTR, Kpad, th);
      la.store(Aim, FB_TSTR, Kpad, th);
    }
    __syncthreads();
    if constexpr (ADAM) {
      if (it == 0 && fin) {
#pragma unroll
        for (int s2 = 0; s2 < U; ++s2) {
          const int u = g * U + s2, i = u >> 1, jj = u & 1;
          const int64_t o = (int64_t)(j0 + wn + jj * 16 + lr) * FC1_N + n0 + wm + i * 16 + 4 * lg;
          pp[s2] = *reinterpret_cast<const float4*>(ad.p + o);
          mm[s2] = *reinterpret_cast<const float4*>(ad.m + o);
          vv[s2] = *reinterpret_cast<const float4*>(ad.v + o);
        }
      }
    }
    const int rn = rows_of(c + G);
    if (rn > 0) {
      lz.load(dzw + (int64_t)(c + G) * MAXB * FC1_N + n0, FC1_N, (rn + 31) & ~31, rn, th);
      la.load(a2w + (int64_t)(c + G) * MAXB * a2s + (j0 - a2c0), a2s, (rn + 31) & ~31, rn, th);
    }
    for (int k0 = 0; k0 < Kpad; k0 += 32) {
      bf16x8 af[SI], bfv[2];
#pragma unroll
      for (int i = 0; i < SI; ++i) {
        const u16* zr = Zim + (k0 + 8 * lg + q) * FB_TSTR + wm + i * 16 + 4 * p;
        af[i] = frag_tr(zr, zr + 4 * FB_TSTR);
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const u16* ar = Aim + (k0 + 8 * lg + q) * FB_TSTR + wn + jj * 16 + 4 * p;
        bfv[jj] = frag_tr(ar, ar + 4 * FB_TSTR);
      }
#pragma unroll
      for (int i = 0; i < SI; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) acc[i][jj] = mfma16(af[i], bfv[jj], acc[i][jj]);
    }
  }
  // exchange: every group stores its partial sub-tiles, then sums the groups' partials of its own
  __syncthreads();
  f32x4* xr = reinterpret_cast<f32x4*>(smem);  // [group][256 threads][S sub-tiles]
#pragma unroll
  for (int u = 0; u < S; ++u) xr[(g * 256 + th) * S + u] = acc[u >> 1][u & 1];
  __syncthreads();
  if (!fin) return;
#pragma unroll
  for (int s2 = 0; s2 < U; ++s2) {
    const int u = g * U + s2, jj = u & 1, i = u >> 1;
    f32x4 sum = xr[th * S + u];
#pragma unroll
    for (int gg = 1; gg < G; ++gg) sum = sum + xr[(gg * 256 + th) * S + u];  // groups in order
    const int64_t o = (int64_t)(j0 + wn + jj * 16 + lr) * FC1_N + n0 + wm + i * 16 + 4 * lg;
    const float4 gv = make_float4(sum[0], sum[1], sum[2], sum[3]);
    if constexpr (ADAM) {
      const AdamCoef cf = adam_coef((float)ad.state[ST_OPT], ad.lr, ad.b1, ad.b2, ad.eps, ad.gscale, ad.rule);
      if (write_grad) *reinterpret_cast<float4*>(gW3 + o) = gv;
      const uint2 sh = adam4(pp[s2], mm[s2], vv[s2], gv, cf);
      *reinterpret_cast<float4*>(ad.p + o) = pp[s2];
      *reinterpret_cast<float4*>(ad.m + o) = mm[s2];
      *reinterpret_cast<float4*>(ad.v + o) = vv[s2];
      *reinterpret_cast<uint2*>(ad.shadow + o) = sh;
    } else {
      *reinterpret_cast<float4*>(gW3 + o) = gv;
    }
  }
}

template <bool ADAM, int G, int NTW = 64>
__global__ void __launch_bounds__(256 * G) fc1_dw3_kg_kernel(const u16* __restrict__ dzw, const u16* __restrict__ a2w,
                                                             int Kw, float* __restrict__ gW3, int tile_base, AdamArgs ad,
                                                             int write_grad, int a2s, int a2c0, CollRole cr) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  if ((int)blockIdx.x < cr.nblk) {  // co-launched xGMI collective (xgmi_role.h)
    coll_role_run(cr, blockIdx.x);
    return;
  }
  fc1_dw3_tile_kg<ADAM, G, NTW>(tile_base + (int)blockIdx.x - cr.nblk, dzw, a2w, Kw, gW3, ad, write_grad, a2s, a2c0,
                                smem);
}

// fc1_bwd: the dgrad tiles and every fc1_wgrad role (local batch) in one launch. The dgrad blocks
// come first (they are the longest and keep the blockIdx -> XCD map their tiles rely on).
__global__ void __launch_bounds__(256) fc1_bwd_kernel(const u16* __restrict__ dz, const u16* __restrict__ a2,
                                                      const u16* __restrict__ h, const float* __restrict__ dlog,
                                                      const u16* __restrict__ w3, u16* __restrict__ g2,
                                                      float* __restrict__ gW3, float* __restrict__ gb3,
                                                      float* __restrict__ gW4, float* __restrict__ gb4, int B, int G,
                                                      int n_dg, int n_small, CollRole cr, u16* __restrict__ a2T,
                                                      u16* __restrict__ dzT) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  // co-launched xGMI collective on the first cr.nblk blocks (a multiple of 8, so the dgrad tiles
  // keep their blockIdx -> XCD map)
  if ((int)blockIdx.x < cr.nblk) {
    coll_role_run(cr, blockIdx.x);
    return;
  }
  const int bx = (int)blockIdx.x - cr.nblk;
  if (bx < n_dg) {
    fc1_dgrad_block(bx, dz, w3, a2, g2, B, G, smem, a2T, dzT);
    return;
  }
  fc1_wgrad_block<false>(bx - n_dg, dz, a2, h, dlog, dz, a2, B, gW3, gb3, gW4, gb4, B, 0, n_small, AdamArgs{}, 1,
                         FC1_K, 0, smem);
}

// ------------------------------------------------------------------------------------------ //
#define MIHVD_MT_SWITCH(MTV, ...)                         \
  switch (MTV) {                                          \
    case 1: { constexpr int MT_ = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int MT_ = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int MT_ = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int MT_ = 4; __VA_ARGS__; } break; \
    case 5: { constexpr int MT_ = 5; __VA_ARGS__; } break; \
    case 6: { constexpr int MT_ = 6; __VA_ARGS__; } break; \
    case 7: { constexpr int MT_ = 7; __VA_ARGS__; } break; \
    default: { constexpr int MT_ = 8; __VA_ARGS__; } break; \
  }

template <typename K>
static void set_max_lds(K kernel, int bytes) {
  (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

void fc1_fwd(const at::Tensor& a2, const at::Tensor& w3bf, at::Tensor& zpart) {
  const int B = a2.size(0);
  TORCH_CHECK(B >= 1 && B <= MAXB, "fc1_fwd: batch must be in [1, 128] (got ", B, ")");
  TORCH_CHECK(a2.dtype() == MIHVD_OP16 && a2.numel() == (int64_t)B * FC1_K && a2.is_contiguous(), "fc1_fwd: a2");
  TORCH_CHECK(w3bf.dtype() == MIHVD_OP16 && w3bf.numel() == (int64_t)FC1_K * FC1_N && w3bf.is_contiguous(), "fc1_fwd: w3");
  TORCH_CHECK(zpart.dtype() == at::kFloat && zpart.numel() == (int64_t)FC1_KS * B * FC1_N, "fc1_fwd: zpart [7][B][1024]");
  const int MT = (B + 15) >> 4;
  const int lds = (FC1_KSL * F1_WSTR + MT * 16 * F1_ASTR) * 2;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  // 8 waves per block (one block per CU: LDS)
  MIHVD_MT_SWITCH(MT, {
    set_max_lds(fc1_fwd_kernel<MT_, 8>, F1_LDS);
    fc1_fwd_kernel<MT_, 8><<<dim3(FC1_N / FC1_NT, FC1_KS), 512, lds, stream>>>(
        (const u16*)a2.data_ptr(), (const u16*)w3bf.data_ptr(), zpart.data_ptr<float>(), B);
  })
}

void head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                  const at::Tensor& labels, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                  int64_t seed, double rate, at::Tensor& h, at::Tensor& dz, at::Tensor& dlog, at::Tensor& stats,
                  int64_t coll, double dz_scale, const c10::optional<at::Tensor>& stats_acc,
                  const c10::optional<at::Tensor>& loss_scale) {
  const int B = h.size(0);
  TORCH_CHECK(zpart.dtype() == at::kFloat && zpart.numel() == (int64_t)FC1_KS * B * FC1_N, "head: zpart");
  TORCH_CHECK(b3.numel() == FC1_N && w4.numel() == FC1_N * 10 && b4.numel() == 10 && w4.dtype() == at::kFloat, "head: params");
  TORCH_CHECK(labels.dtype() == at::kLong, "head: labels must be int64");
  TORCH_CHECK(h.dtype() == MIHVD_OP16 && h.numel() == (int64_t)B * FC1_N && dz.numel() == h.numel(), "head: h/dz");
  TORCH_CHECK(dlog.numel() == B * 10 && stats.numel() == B * 2, "head: dlog/stats");
  TORCH_CHECK(rate >= 0.0 && rate < 1.0, "head: dropout rate");
  float* acc = nullptr;
  if (stats_acc.has_value() && stats_acc->defined()) {
    TORCH_CHECK(stats_acc->is_cuda() && stats_acc->dtype() == at::kFloat && stats_acc->is_contiguous() &&
                    stats_acc->numel() == B * 2, "head: stats_acc must be a contiguous fp32 [B][2] device tensor");
    acc = stats_acc->data_ptr<float>();
  }
  const int* rp = nullptr;
  int n_pool = labels.numel();
  if (rows.has_value() && rows->defined()) rp = rows->data_ptr<int>();
  else TORCH_CHECK(n_pool >= B, "head: labels shorter than the batch");
  int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  const uint32_t thresh = (uint32_t)(rate * 16777216.0);
  const float keep_scale = (float)(1.0 / (1.0 - rate));
  const float* lsp = nullptr;
  if (loss_scale.has_value() && loss_scale->defined()) {
    TORCH_CHECK(loss_scale->is_cuda() && loss_scale->dtype() == at::kFloat && loss_scale->numel() == 2,
                "head: loss_scale must be the float32 device pair [scale, found_nonfinite]");
    TORCH_CHECK(dz_scale == 1.0, "head: a device loss scale replaces dz_scale");
    lsp = loss_scale->data_ptr<float>();
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const CollRole cr = xgmi_role_lookup(coll);
  head_kernel<<<B + cr.nblk, 256, 0, stream>>>(zpart.data_ptr<float>(), b3.data_ptr<float>(), w4.data_ptr<float>(),
                                               b4.data_ptr<float>(), labels.data_ptr<int64_t>(), rp, n_pool, sp,
                                               (uint32_t)seed, thresh, keep_scale, (float)(keep_scale * dz_scale),
                                               (u16*)h.data_ptr(),
                                               (u16*)dz.data_ptr(), dlog.data_ptr<float>(), stats.data_ptr<float>(), B,
                                               cr, acc, lsp);
}

// roles: bit 0 = the dW3 tiles, bit 1 = the small reductions (db3, dW4, db4). dW3 multiplies dz_w3^T a2_w3 over their rows: the local dz/a2 by default, or the
// all-gathered factors of every rank (data-parallel "factor gather": dW3 = sum over all samples,
// exactly what the allreduce of per-rank dW3 would produce, for a fraction of the bytes).
static void fc1_wgrad_launch(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog,
                             at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, int64_t roles,
                             const c10::optional<at::Tensor>& dz_w3, const c10::optional<at::Tensor>& a2_w3,
                             const AdamArgs* ad, bool write_grad, int64_t jt_lo, int64_t jt_hi, int64_t coll) {
  const int B = dz.size(0);
  TORCH_CHECK(B >= 1 && B <= MAXB, "fc1_wgrad: batch");
  TORCH_CHECK(dz.dtype() == MIHVD_OP16 && dz.numel() == (int64_t)B * FC1_N, "fc1_wgrad: dz");
  TORCH_CHECK(a2.numel() == (int64_t)B * FC1_K && a2.dtype() == MIHVD_OP16, "fc1_wgrad: a2");
  TORCH_CHECK(h.numel() == (int64_t)B * FC1_N && h.dtype() == MIHVD_OP16 && dlog.numel() == B * 10, "fc1_wgrad: h/dlog");
  TORCH_CHECK(gW3.numel() == (int64_t)FC1_K * FC1_N && gW3.dtype() == at::kFloat && gW3.is_contiguous(), "fc1_wgrad: gW3");
  TORCH_CHECK(gb3.numel() == FC1_N && gW4.numel() == FC1_N * 10 && gb4.numel() == 10, "fc1_wgrad: fc grads");
  TORCH_CHECK(roles >= 1 && roles <= 3, "fc1_wgrad: roles must be 1, 2 or 3");
  const u16* dzw = (const u16*)dz.data_ptr();
  const u16* a2w = (const u16*)a2.data_ptr();
  int a2s = FC1_K, a2c0 = 0;
  int Kw = B;
  if (dz_w3.has_value() && dz_w3->defined()) {
    TORCH_CHECK(a2_w3.has_value() && a2_w3->defined(), "fc1_wgrad: dz_w3 and a2_w3 go together");
    Kw = dz_w3->size(0);
    TORCH_CHECK(dz_w3->dtype() == MIHVD_OP16 && dz_w3->numel() == (int64_t)Kw * FC1_N && dz_w3->is_contiguous(),
                "fc1_wgrad: dz_w3 [K][1024] bf16");
    TORCH_CHECK(a2_w3->dtype() == MIHVD_OP16 && a2_w3->is_contiguous() && a2_w3->numel() % Kw == 0,
                "fc1_wgrad: a2_w3 [K][3136] (or [K][C] columns of the row-tile range) bf16");
    a2s = (int)(a2_w3->numel() / Kw);
    if (a2s != FC1_K) {
      // only the columns of the dW3 row tiles [jt_lo, jt_hi), starting at column jt_lo * 64
      a2c0 = (int)jt_lo * 64;
      TORCH_CHECK(a2s % 8 == 0 && a2s >= (int)(jt_hi - jt_lo) * 64,
                  "fc1_wgrad: a2_w3 column slice must cover the row-tile range (and be a multiple of 8)");
    }
    TORCH_CHECK(Kw >= 1 && Kw <= 65536, "fc1_wgrad: K");
    dzw = (const u16*)dz_w3->data_ptr();
    a2w = (const u16*)a2_w3->data_ptr();
  }
  int role = debug_role_only();  // kbench: 0 = dW3 tiles only, 1 = small reductions only
  if (role == 0) roles &= 1;
  if (role == 1) roles &= 2;
  TORCH_CHECK(0 <= jt_lo && jt_lo <= jt_hi && jt_hi <= FC1_K / 64, "fc1_wgrad: dW3 row-tile range must lie in [0, 49]");
  const int n_small = (roles & 2) ? FB_TOTAL - FB_WGRAD : 0;
  const int tile_base = (int)jt_lo * (FC1_N / 64);
  const CollRole cr = xgmi_role_lookup(coll);
  const int grid = n_small + ((roles & 1) ? (int)(jt_hi - jt_lo) * (FC1_N / 64) : 0) + cr.nblk;
  if (grid == 0) return;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const u16 *pdz = (const u16*)dz.data_ptr(), *pa2 = (const u16*)a2.data_ptr(), *ph = (const u16*)h.data_ptr();
  // dW3 tiles alone over a K of two or more 128-row chunks (all-gathered factors): the K-split
  // group tiles, 2 groups, or 4 from 4 chunks on (the 4- and 8-rank factors)
  constexpr int kg4_from = 4;
  if (roles == 1 && Kw > MAXB) {
    const int nch = (Kw + MAXB - 1) / MAXB;
    auto run = [&](auto kt, auto ka, int groups) {
      const int lds = groups * FB_LDS_WG;
      if (ad != nullptr) {
        set_max_lds(ka, lds);
        ka<<<grid, 256 * groups, lds, stream>>>(dzw, a2w, Kw, gW3.data_ptr<float>(), tile_base, *ad,
                                                write_grad ? 1 : 0, a2s, a2c0, cr);
      } else {
        set_max_lds(kt, lds);
        kt<<<grid, 256 * groups, lds, stream>>>(dzw, a2w, Kw, gW3.data_ptr<float>(), tile_base, AdamArgs{}, 1,
                                                a2s, a2c0, cr);
      }
    };
    // four groups only for a row slice that fits the CUs one block each (the sharded optimizer's
    // 1/N of the rows): over all 784 tiles the 1024-thread blocks cut occupancy (measured 22.3 ->
    // 29.9 us at the 8-rank K), over the 8-rank slice they win (7.7 -> 7.2 us, with Adam 12.8 ->
    // 11.4), over the 4-rank slice (13 row tiles, K = 400) dW3 + Adam 11.2 -> 9.6 us
    const int tiles = (int)(jt_hi - jt_lo) * (FC1_N / 64);
    const int ncu = device_cu_count();
    // 32-feature tiles (twice the blocks, each with half the MFMA work and half the Adam epilogue)
    // when they still fit the CUs one block each: the 8-rank slice dW3 7.2 -> 6.3 us, dW3 + Adam
    // 11.4 -> 9.0 us
    if (nch >= kg4_from && 2 * tiles + cr.nblk <= ncu) {
      const int grid32 = 2 * tiles + cr.nblk;
      const int lds = 4 * FB_LDS_WG;
      const int tb32 = (int)jt_lo * (FC1_N / 32);
      if (ad != nullptr) {
        set_max_lds(fc1_dw3_kg_kernel<true, 4, 32>, lds);
        fc1_dw3_kg_kernel<true, 4, 32><<<grid32, 1024, lds, stream>>>(dzw, a2w, Kw, gW3.data_ptr<float>(), tb32, *ad,
                                                                      write_grad ? 1 : 0, a2s, a2c0, cr);
      } else {
        set_max_lds(fc1_dw3_kg_kernel<false, 4, 32>, lds);
        fc1_dw3_kg_kernel<false, 4, 32><<<grid32, 1024, lds, stream>>>(dzw, a2w, Kw, gW3.data_ptr<float>(), tb32,
                                                                       AdamArgs{}, 1, a2s, a2c0, cr);
      }
      return;
    }
    if (nch >= kg4_from && tiles + cr.nblk <= ncu)
      run(fc1_dw3_kg_kernel<false, 4>, fc1_dw3_kg_kernel<true, 4>, 4);
    else run(fc1_dw3_kg_kernel<false, 2>, fc1_dw3_kg_kernel<true, 2>, 2);
    return;
  }
  if (ad != nullptr) {
    fc1_wgrad_kernel<true><<<grid, 256, FB_LDS_WG, stream>>>(
        pdz, pa2, ph, dlog.data_ptr<float>(), dzw, a2w, Kw, gW3.data_ptr<float>(), gb3.data_ptr<float>(),
        gW4.data_ptr<float>(), gb4.data_ptr<float>(), B, tile_base, n_small, *ad, write_grad ? 1 : 0, a2s, a2c0, cr);
  } else {
    fc1_wgrad_kernel<false><<<grid, 256, FB_LDS_WG, stream>>>(
        pdz, pa2, ph, dlog.data_ptr<float>(), dzw, a2w, Kw, gW3.data_ptr<float>(), gb3.data_ptr<float>(),
        gW4.data_ptr<float>(), gb4.data_ptr<float>(), B, tile_base, n_small, AdamArgs{}, 1, a2s, a2c0, cr);
  }
}

void fc1_wgrad(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog, at::Tensor& gW3,
               at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, int64_t roles, const c10::optional<at::Tensor>& dz_w3,
               const c10::optional<at::Tensor>& a2_w3, int64_t jt_lo, int64_t jt_hi, int64_t coll) {
  fc1_wgrad_launch(dz, a2, h, dlog, gW3, gb3, gW4, gb4, roles, dz_w3, a2_w3, nullptr, true, jt_lo, jt_hi, coll);
}

// fc1_wgrad with the Adam update of dense/kernel fused into the dW3 tiles (see the kernel). p3, m3,
// v3 (fp32) and shadow3 (bf16) are the dense/kernel segments of the flat buffers (indexed by W3 row:
// only the rows of the tiles [jt_lo, jt_hi) are touched); state is the device step state (the
// optimizer step t is read from it; this op does not advance it).
void fc1_wgrad_adam(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog,
                    at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, int64_t roles,
                    const c10::optional<at::Tensor>& dz_w3, const c10::optional<at::Tensor>& a2_w3, at::Tensor& p3,
                    at::Tensor& m3, at::Tensor& v3, at::Tensor& shadow3, const at::Tensor& state, double lr, double b1,
                    double b2, double eps, double grad_scale, int64_t rule, bool write_grad, int64_t jt_lo,
                    int64_t jt_hi, int64_t coll) {
  const int64_t n = (int64_t)FC1_K * FC1_N;
  for (const at::Tensor* t : {&p3, &m3, &v3})
    TORCH_CHECK(t->dtype() == at::kFloat && t->numel() == n && t->is_contiguous(), "fc1_wgrad_adam: p3/m3/v3 fp32 [3136*1024]");
  TORCH_CHECK(shadow3.dtype() == MIHVD_OP16 && shadow3.numel() == n && shadow3.is_contiguous(), "fc1_wgrad_adam: shadow3");
  TORCH_CHECK(state.dtype() == at::kLong && state.numel() >= ST_WORDS, "fc1_wgrad_adam: state");
  for (const at::Tensor* t : {&p3, &m3, &v3, &shadow3})
    TORCH_CHECK(((uintptr_t)t->data_ptr() & 15) == 0, "fc1_wgrad_adam: 16-byte aligned segments required");
  AdamArgs ad{p3.data_ptr<float>(), m3.data_ptr<float>(), v3.data_ptr<float>(), (u16*)shadow3.data_ptr(),
              state.data_ptr<int64_t>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale, (int)rule};
  fc1_wgrad_launch(dz, a2, h, dlog, gW3, gb3, gW4, gb4, roles, dz_w3, a2_w3, &ad, write_grad, jt_lo, jt_hi, coll);
}

// dgrad: g2 = (a2 > 0) * dz.W3^T in bf16, the gradient conv2_bwd routes through the pool argmax.
void fc1_dgrad(const at::Tensor& dz, const at::Tensor& w3bf, const at::Tensor& a2, at::Tensor& g2) {
  const int B = dz.size(0);
  TORCH_CHECK(B >= 1 && B <= MAXB, "fc1_dgrad: batch");
  TORCH_CHECK(dz.dtype() == MIHVD_OP16 && dz.numel() == (int64_t)B * FC1_N && dz.is_contiguous(), "fc1_dgrad: dz");
  TORCH_CHECK(w3bf.dtype() == MIHVD_OP16 && w3bf.numel() == (int64_t)FC1_K * FC1_N && w3bf.is_contiguous(), "fc1_dgrad: w3");
  TORCH_CHECK(a2.dtype() == MIHVD_OP16 && a2.numel() == (int64_t)B * FC1_K && a2.is_contiguous(), "fc1_dgrad: a2");
  TORCH_CHECK(g2.dtype() == MIHVD_OP16 && g2.numel() == (int64_t)B * FC1_K && g2.is_contiguous(), "fc1_dgrad: g2");
  const int G = (B + DG_ROWS - 1) / DG_ROWS;
  const int grid = 8 * ((DG_JT + 7) / 8) * G;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  set_max_lds(fc1_dgrad_kernel, DG_LDS);
  fc1_dgrad_kernel<<<grid, 256, DG_LDS, stream>>>((const u16*)dz.data_ptr(), (const u16*)w3bf.data_ptr(),
                                                   (const u16*)a2.data_ptr(), (u16*)g2.data_ptr(), B, G);
}

// fc1_wgrad (every role, local batch) + fc1_dgrad in one launch (fc1_bwd_kernel).
// roles as fc1_wgrad: bit 0 = the dW3 tiles, bit 1 = db3 / dW4 / db4.
void fc1_bwd(const at::Tensor& dz, const at::Tensor& a2, const at::Tensor& h, const at::Tensor& dlog,
             const at::Tensor& w3bf, at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4, at::Tensor& g2,
             int64_t roles, int64_t coll, const c10::optional<at::Tensor>& a2T,
             const c10::optional<at::Tensor>& dzT) {
  TORCH_CHECK(roles >= 1 && roles <= 3, "fc1_bwd: roles must be 1, 2 or 3");
  const int B = dz.size(0);
  TORCH_CHECK(B >= 1 && B <= MAXB, "fc1_bwd: batch");
  TORCH_CHECK(dz.dtype() == MIHVD_OP16 && dz.numel() == (int64_t)B * FC1_N && dz.is_contiguous(), "fc1_bwd: dz");
  TORCH_CHECK(a2.dtype() == MIHVD_OP16 && a2.numel() == (int64_t)B * FC1_K && a2.is_contiguous(), "fc1_bwd: a2");
  TORCH_CHECK(h.numel() == (int64_t)B * FC1_N && h.dtype() == MIHVD_OP16 && dlog.numel() == B * 10, "fc1_bwd: h/dlog");
  TORCH_CHECK(w3bf.dtype() == MIHVD_OP16 && w3bf.numel() == (int64_t)FC1_K * FC1_N && w3bf.is_contiguous(), "fc1_bwd: w3");
  TORCH_CHECK(gW3.numel() == (int64_t)FC1_K * FC1_N && gW3.dtype() == at::kFloat && gW3.is_contiguous(), "fc1_bwd: gW3");
  TORCH_CHECK(gb3.numel() == FC1_N && gW4.numel() == FC1_N * 10 && gb4.numel() == 10, "fc1_bwd: fc grads");
  TORCH_CHECK(g2.dtype() == MIHVD_OP16 && g2.numel() == (int64_t)B * FC1_K && g2.is_contiguous(), "fc1_bwd: g2");
  const int G = (B + DG_ROWS - 1) / DG_ROWS;
  const int n_dg = 8 * ((DG_JT + 7) / 8) * G;
  const int n_small = (roles & 2) ? FB_TOTAL - FB_WGRAD : 0;
  CollRole cr = xgmi_role_lookup(coll);
  TORCH_CHECK(cr.nblk % 8 == 0, "fc1_bwd: a co-launched collective needs a multiple of 8 blocks (XCD map)");
  const int grid = cr.nblk + n_dg + n_small + ((roles & 1) ? FB_WGRAD : 0);
  u16 *pa2T = nullptr, *pdzT = nullptr;
  if (a2T.has_value() && a2T->defined()) {
    TORCH_CHECK(dzT.has_value() && dzT->defined(), "fc1_bwd: a2T and dzT go together");
    TORCH_CHECK(a2T->dtype() == MIHVD_OP16 && a2T->numel() == (int64_t)FC1_K * FT_KP && a2T->is_contiguous(),
                "fc1_bwd: a2T must be bf16 [3136][128]");
    TORCH_CHECK(dzT->dtype() == MIHVD_OP16 && dzT->numel() == (int64_t)FC1_N * FT_KP && dzT->is_contiguous(),
                "fc1_bwd: dzT must be bf16 [1024][128]");
    pa2T = (u16*)a2T->data_ptr();
    pdzT = (u16*)dzT->data_ptr();
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  set_max_lds(fc1_bwd_kernel, DG_LDS);
  fc1_bwd_kernel<<<grid, 256, DG_LDS, stream>>>(
      (const u16*)dz.data_ptr(), (const u16*)a2.data_ptr(), (const u16*)h.data_ptr(), dlog.data_ptr<float>(),
      (const u16*)w3bf.data_ptr(), (u16*)g2.data_ptr(), gW3.data_ptr<float>(), gb3.data_ptr<float>(),
      gW4.data_ptr<float>(), gb4.data_ptr<float>(), B, G, n_dg, n_small, cr, pa2T, pdzT);
}

MIHVD_OPNS_END
