// Backward convolutions of the MNIST CNN.
//
// conv2_bwd (one launch, 512-thread blocks, two roles):
//   * The routed conv2 output gradient dY2 is built on the fly in LDS from g2 (fc1_dgrad's bf16
//     output, already masked with conv2's pooled ReLU) scattered through the argmax indices idx2
//     (4 co per lane -> four 8-byte LDS writes). dY2 never exists in HBM.
//   * dgrad (one block per image): dA1 = full correlation of dY2 with W2 as an implicit GEMM
//     (K = 25 taps x 64 channels), W2 resident in LDS (100 KB, swizzled), output features on the
//     MFMA row axis and one image row per pixel tile; conv1's pooled ReLU mask is applied in the
//     epilogue -> g1 (bf16). db2 is reduced here.
//   * wgrad (kernel row kh x group of 4 images): dW2 as an MFMA GEMM over pixels with both operands
//     read by ds_read_b64_tr_b16 from natural NHWC images; two 4-wave groups take two images each
//     and are summed in LDS; one fp32 partial slab per block (deterministic, no atomics).
//   The dgrad role then computes conv1's weight gradient for its image from g1 still on chip: dW1/db1
//   as an MFMA GEMM over full-resolution pixels (the routed gradient is scattered into LDS,
//   im2col(x) is read from kw-shifted image copies).
// conv2_wgrad_reduce: dW2 = sum of the wgrad slabs.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"
#include "w3_tail.h"
#include "xgmi_role.h"

MIHVD_OPNS_BEGIN

constexpr int CB_IPB = 4;               // images per wgrad block (2 per wave group)
constexpr int CB_KQ = 4;                // fc1 dgrad split-K slabs
// The wgrad dY2 image (128-B pixel rows, 16 groups of 8 B) is XOR-swizzled on its 8-byte groups
// so the transposed reads (ds_read_b64_tr_b16, 32-lane groups) hit distinct banks.
__device__ __forceinline__ int swd(int r) { return 4 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }
// dgrad LDS: W2 [800][64] | D [326][64], both unpadded 128-B rows whose eight 16-B chunks are
// XOR-swizzled with the row index (chunk' = chunk ^ (row & 7)). With output tiles of 16
// consecutive pixels (one image row, x = 0..15) every ds_read_b128 lane group of the A and B
// fragment reads hits 64 distinct banks (checked with a bank model of the lane groups).
constexpr int CB_DG_W = 800 * 64;
constexpr int CB_DG_D = 326 * 64;                                  // 18 x 18 halo image + 2 spare rows
// + conv1-tail operands staged with the dgrad operands, outside the W2 / dY2 images: the five
// kw-shifted bf16 input images [5][32][32], a zero chunk and the bias fold slots (db2 [8 waves][16]
// float4, db1 [8 waves][4 lg][8]), 13,328 B. The launch adds the kernel's static LDS (the
// co-launched roles) and checks the sum against the CU's 163,840 B.
constexpr int CB_X_OFF = CB_DG_W + CB_DG_D;                        // elements
constexpr int CB_X_LDS = (5 * 32 * 32 + 8) * 2 + (512 + 256) * 4;
constexpr int CB_DG_LDS = (CB_DG_W + CB_DG_D) * 2 + CB_X_LDS;      // 157,456 B
static_assert(CB_DG_LDS <= 163840 - 1024, "dgrad LDS fits one CU with room for static LDS");
__device__ __forceinline__ int swz64(int row, int chunk) { return row * 64 + 8 * (chunk ^ (row & 7)); }
// wgrad LDS per wave group: A [325][32] | Dm [197][64]
constexpr int CB_WG_A = 325 * 32;
constexpr int CB_WG_D = 197 * 64;
constexpr int CB_WG_GRP = CB_WG_A + CB_WG_D;                       // elements
constexpr int CB_WG_LDS = 2 * CB_WG_GRP * 2;                       // 98,336 B
constexpr int CB_LDS = CB_DG_LDS > CB_WG_LDS ? CB_DG_LDS : CB_WG_LDS;

// ------------------------------------------------------------------------------------------ //
// Fused conv1 weight gradient (tail of the conv2 dgrad role, one image per block): dW1/db1 -> atomics.
//
// It is an MFMA GEMM over the full-resolution pixels of the image:
//     dW1^T[co][tap] = sum_pix dY1^T[co][pix] * im2col(x)[pix][tap]      (M = 32, N = 25 -> 32)
// with K = 28 rows x 32 columns (columns 28..31 are dummy pixels whose dY1 row is the zero row).
//   * dY1 ([785][40] bf16, pixel rows) is scattered from the pooled gradient g1 (the dgrad
//     epilogue's registers, never re-read from HBM) through the argmax slots idx1 (each pooling window writes its four sub-pixels, value or zero), so every pixel
//     row is written once and only the zero row needs clearing; it is read by transposed LDS
//     reads (ds_read_b64_tr_b16) as the A operand.
//   * im2col(x) is never built: the B fragment of tap (kh, kw) for 8 consecutive pixels of a row
//     is 8 consecutive elements of the zero-padded image row y + kh starting at column x0 + kw.
//     Five copies of the bf16 image shifted by kw = 0..4 make that one aligned ds_read_b128.
//   * the eight waves split K (image rows w, w+8, ...) and are summed through LDS before the atomics.
// ------------------------------------------------------------------------------------------ //
// Per-image partial row of the small conv gradients, reduced (in a fixed order: deterministic, no
// atomics contending for the same few cache lines) by conv2_wgrad_reduce.
constexpr int CP_DB1 = 800, CP_DB2 = 832, CP_W = 896;  // [dW1 (800) | db1 (32) | db2 (64)]
constexpr int C1_DSTR = 40;                          // dY1 row stride (32 co + 8 pad)
constexpr int C1_DY = 785 * C1_DSTR;                 // elements; row 784 = zeros
constexpr int C1_XS = 32 * 32;                       // one shifted bf16 image copy [32][32]
static_assert(C1_DY * 2 <= CB_DG_W * 2, "dY1 fits in the dead W2 image");
static_assert(8 * 64 * 16 * 4 <= CB_DG_D * 2, "the GEMM partials fit in the dead dY2 image");



struct DyItem {
  uint2 g;       // 4 bf16 pooled gradients (already masked by conv2's pooled ReLU)
  uint32_t idx;  // 4 argmax slots
};

// Loads for one dY2 build item: 4 consecutive channels of one pooling window of image b.
__device__ __forceinline__ DyItem load_dy_item(const u16* __restrict__ g2, const uint8_t* __restrict__ idx2, int b,
                                               int e) {
  DyItem it;
  it.g = *reinterpret_cast<const uint2*>(g2 + (int64_t)b * 3136 + e);
  it.idx = *reinterpret_cast<const uint32_t*>(idx2 + (int64_t)b * 3136 + e);
  return it;
}

__device__ __forceinline__ void finish_dy_item(const DyItem& it, u16 g[4], int d[4], float gf[4]) {
  g[0] = (u16)(it.g.x & 0xffff);
  g[1] = (u16)(it.g.x >> 16);
  g[2] = (u16)(it.g.y & 0xffff);
  g[3] = (u16)(it.g.y >> 16);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    gf[c] = bf2f(g[c]);
    d[c] = (it.idx >> (8 * c)) & 3;
  }
}

// Barrier of the conv roles' eight waves. With streamer waves in the block (TAIL_ADAM launches
// of 512 + 64 * SW threads, below) a hardware s_barrier would also wait for the streamers, so
// the eight conv waves meet on an LDS counter instead: each wave adds 1 after its LDS accesses
// have completed (workgroup release) and waits until the counter reaches 8 x its barrier count.
// Set (atomic OR) by a ConvBarrier whose bounded wait ran out: the conv gradients of that launch
// are invalid. Read and cleared by conv_barrier_error() (the trainer's check after every replay).
__device__ unsigned g_conv_barrier_err = 0;

template <bool SWB>
struct ConvBarrier {
  unsigned* ctr;
  unsigned gen = 0;
  __device__ __forceinline__ void sync() {
    if constexpr (!SWB) {
      __syncthreads();
    } else {
      gen += 8;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // bounded: a broken count ends the wait (wrong results, not a hung GPU) after ~30 ms, and
      // raises the device error word so the host reports it instead of training on it
      int spin = 0;
      for (; spin < (1 << 20) && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < gen; ++spin)
        __builtin_amdgcn_s_sleep(1);
      if (spin == (1 << 20)) __hip_atomic_fetch_or(&g_conv_barrier_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
  }
};

// Stores of the outputs that the reduction reads. WT (the folded reduction, below): write-through
// (sc1) so that another XCD's reduction can read them after the arrival counter with no release.
__device__ __forceinline__ void out_store1(float* p, float v, bool wt) {
  if (wt) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

template <bool SWB>
__device__ __forceinline__ void conv2_bwd_block(
    const u16* __restrict__ g2, const uint8_t* __restrict__ idx2,
    const u16* __restrict__ a1, const u16* __restrict__ w2bf, const float* __restrict__ x, const int* __restrict__ rows,
    int n_pool, const int64_t* __restrict__ state, const uint8_t* __restrict__ idx1, u16* __restrict__ g1,
    float* __restrict__ slab, float* __restrict__ cpart, int B, int n_dgrad, int dbg_exit, int bx,
    ConvBarrier<SWB>& bar, bool wt = false) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  if (bx < n_dgrad) {
    // ===================================================================== dgrad: image b
    const int b = bx;
    u16* Ws = smem;              // [800][64] swizzled, row = kk*32 + ci, cols = co
    u16* D = smem + CB_DG_W;     // [326][64] swizzled padded dY2 image (pixel = row)
    // Issue every load of the block first: W2 (direct to LDS), 2 dY2 items and the epilogue's
    // conv1 pooled-ReLU mask.
    DyItem items[2];
    int ie[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = min(t + 512 * k, 783);
      ie[k] = t + 512 * k;
      items[k] = load_dy_item(g2, idx2, b, (i >> 4) * 64 + (i & 15) * 4);
    }
    glds_swz128<512>(w2bf, Ws, 800 * 8, t);  // W2 straight into its swizzled LDS image
    // output tiles: image row y = wave and wave + 8 (rows 14, 15 are dummies), pixel x = lr
    // (x = 14, 15 dummies); lane holds ci 16*nt + 4*lg .. +3 of that pixel.
    uint2 amask[2][2];
    uint32_t dsel[2][2];  // conv1 pool argmax slots of the same 4 channels (fused conv1 wgrad)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int y = min(wave + 8 * i, 13), xx = min(lr, 13);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int64_t o = ((int64_t)b * 196 + y * 14 + xx) * 32 + nt * 16 + 4 * lg;
        amask[i][nt] = *reinterpret_cast<const uint2*>(a1 + o);
        dsel[i][nt] = *reinterpret_cast<const uint32_t*>(idx1 + o);
      }
    }
    // the input image for conv1's weight gradient: 2 of the [32][32] zero-padded positions each
    float xv[2];
    {
      int row = b;
      if (rows != nullptr) {
        const int64_t step = state ? state[ST_FWD] : 0;
        row = rows[(int)((step * (int64_t)B + b) % n_pool)];
      }
      const float* xi = x + (int64_t)row * 784;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = t + 512 * k;
        const int gy = (i >> 5) - 2, gx = (i & 31) - 2;
        const bool in = gy >= 0 && gy < 28 && gx >= 0 && gx < 28;
        xv[k] = mask_f(xi[in ? gy * 28 + gx : 0], in);
      }
    }
    // zero the halo pixels (interior pixels are fully written by the scatter); rows 324, 325 are
    // only read by dummy output columns, whose results are discarded
    for (int i = t; i < 324 * 8; i += 512) {
      const int pix = i >> 3, c = i & 7;
      const int y = pix / 18, x = pix - y * 18;
      if (y < 2 || y >= 16 || x < 2 || x >= 16) *reinterpret_cast<uint4*>(D + swz64(pix, c)) = make_uint4(0, 0, 0, 0);
    }
    float db[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (ie[k] < 784) {
        u16 g[4];
        int d[4];
        float gf[4];
        finish_dy_item(items[k], g, d, gf);
#pragma unroll
        for (int c = 0; c < 4; ++c) db[c] += gf[c];
        const int win = ie[k] >> 4, co4 = (ie[k] & 15) * 4;
        const int py = win / 7, px = win - py * 7;
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          const int pix = (2 * py + (dd >> 1) + 2) * 18 + 2 * px + (dd & 1) + 2;
          const uint32_t lo = (uint32_t)(d[0] == dd ? g[0] : 0) | ((uint32_t)(d[1] == dd ? g[1] : 0) << 16);
          const uint32_t hi = (uint32_t)(d[2] == dd ? g[2] : 0) | ((uint32_t)(d[3] == dd ? g[3] : 0) << 16);
          *reinterpret_cast<uint2*>(D + swz64(pix, co4 >> 3) + (co4 & 7)) = make_uint2(lo, hi);
        }
      }
    }
    // The epilogue / conv1-tail operands must have landed here, with the staging loads: left to
    // itself the compiler sinks these loads to their first use after the GEMM and exposes their
    // full latency there.
    // conv1 tail operands: the five kw-shifted bf16 copies of the zero-padded input image,
    // Xs[kw][r][c] = P[r][c + kw] with P = x padded by 2 (columns 32..35 of P are zero)
    u16* Xs = smem + CB_X_OFF;
    u16* Zc = Xs + 5 * C1_XS;  // zero chunk (dummy taps)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = t + 512 * k, r = i >> 5, col = i & 31;
      const u16 v = f2bf(xv[k]);
#pragma unroll
      for (int kw = 0; kw < 5; ++kw)
        if (col >= kw) Xs[kw * C1_XS + r * 32 + col - kw] = v;
    }
    if (t < 320) {  // the 10 entries per row that read P's zero columns: (kw, c) with c + kw >= 32
      const int r = t / 10, e = t - r * 10;
      const int kw = e < 1 ? 1 : e < 3 ? 2 : e < 6 ? 3 : 4;
      const int c = 32 - kw + (e - (kw * (kw - 1)) / 2);
      Xs[kw * C1_XS + r * 32 + c] = 0;
    } else if (t == 320) {
      *reinterpret_cast<uint4*>(Zc) = make_uint4(0, 0, 0, 0);
    }
    bar.sync();
    if (dbg_exit == 1) return;  // profiling: staging only
    // GEMM: rows = ci (2 tiles), cols = 16 pixels of image row y, K = (kh, kw, co) = 1600.
    // Waves 6, 7 compute a dummy second tile (no guard on MFMAs).
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pix0[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) pix0[i] = (min(wave + 8 * i, 13) + 4) * 18 + lr + 4;  // <= 325
#pragma unroll 5
    for (int kk = 0; kk < 25; ++kk) {
      const int kh = kk / 5, kw = kk - kh * 5;
      const int toff = kh * 18 + kw;
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        const int c = ch * 4 + lg;
        const bf16x8 w0 = frag_ld128(Ws + swz64(kk * 32 + lr, c));
        const bf16x8 w1 = frag_ld128(Ws + swz64(kk * 32 + 16 + lr, c));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const bf16x8 bx = frag_ld128(D + swz64(pix0[i] - toff, c));
          acc[i][0] = mfma16(w0, bx, acc[i][0]);
          acc[i][1] = mfma16(w1, bx, acc[i][1]);
        }
      }
    }
    if (dbg_exit == 2 && acc[0][0][0] == 12345.f) g1[0] = 0;  // profiling: keep the GEMM, skip the rest
    if (dbg_exit == 2) return;
    // Epilogue: conv1's pooled-ReLU mask and bf16 rounding -> g1 (kept on chip; written to HBM
    // only when the caller asks for it, e.g. numerics tests).
    uint2 gq[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool valid = wave + 8 * i < 14 && lr < 14;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint2 av = amask[i][nt];
        const float m0 = bf2f((u16)(av.x & 0xffff)) > 0.f ? acc[i][nt][0] : 0.f;
        const float m1 = bf2f((u16)(av.x >> 16)) > 0.f ? acc[i][nt][1] : 0.f;
        const float m2 = bf2f((u16)(av.y & 0xffff)) > 0.f ? acc[i][nt][2] : 0.f;
        const float m3 = bf2f((u16)(av.y >> 16)) > 0.f ? acc[i][nt][3] : 0.f;
        const uint2 v = pack4bf(m0, m1, m2, m3);
        gq[i][nt] = make_uint2(valid ? v.x : 0u, valid ? v.y : 0u);
        if (g1 != nullptr && valid)
          *reinterpret_cast<uint2*>(g1 + ((int64_t)b * 196 + (wave + 8 * i) * 14 + lr) * 32 + nt * 16 + 4 * lg) = v;
      }
    }
    if (dbg_exit == 3) return;  // profiling: no conv1 tail
    // ---- fused conv1 weight gradient (see conv1 section below for the GEMM layout)
    bar.sync();  // W2 and dY2 images are dead: reuse their LDS
    if (dbg_exit == 7) return;  // profiling: conv1 tail cut after its first barrier
    u16* Dy = smem;                                          // [785][40] full-resolution dY1
    float* red = reinterpret_cast<float*>(Zc + 8);           // [8 waves][16] float4 db2 | [8 waves][4 lg][8] db1
    float* red1 = red + 512;
    float d1[8];                                             // db1 partial: (nt, i) channel 16nt+4lg+i
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int y = min(wave + 8 * i, 13);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const uint2 v = gq[i][nt];
        const u16 g[4] = {(u16)(v.x & 0xffff), (u16)(v.x >> 16), (u16)(v.y & 0xffff), (u16)(v.y >> 16)};
#pragma unroll
        for (int c = 0; c < 4; ++c) d1[nt * 4 + c] = (i == 0 ? 0.f : d1[nt * 4 + c]) + bf2f(g[c]);
        if (wave + 8 * i < 14 && lr < 14) {
          int d[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) d[c] = (dsel[i][nt] >> (8 * c)) & 3;
#pragma unroll
          for (int dd = 0; dd < 4; ++dd) {
            const int pix = (2 * y + (dd >> 1)) * 28 + 2 * lr + (dd & 1);
            const uint32_t lo = (uint32_t)(d[0] == dd ? g[0] : 0) | ((uint32_t)(d[1] == dd ? g[1] : 0) << 16);
            const uint32_t hi = (uint32_t)(d[2] == dd ? g[2] : 0) | ((uint32_t)(d[3] == dd ? g[3] : 0) << 16);
            *reinterpret_cast<uint2*>(Dy + pix * C1_DSTR + nt * 16 + 4 * lg) = make_uint2(lo, hi);
          }
        }
      }
    }
    if (dbg_exit == 8) return;  // profiling: ... after the dY1 scatter stores
    // db1: sum the 16 pixels (lanes lr = one DPP row) of each lane group, then one slot per (wave, lg)
#pragma unroll
    for (int c = 0; c < 8; ++c) d1[c] = row_sum16(d1[c]);
    if (lr == 0) {
#pragma unroll
      for (int c = 0; c < 8; ++c) red1[(wave * 4 + lg) * 8 + c] = d1[c];
    }
    // db2: lanes l, l+16, l+32, l+48 of a wave hold the same channel group (t & 15): fold them with
    // two shuffles, then one slot per (wave, group), so the final sum is 8 terms, not 32
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      db[c] += __shfl_xor(db[c], 16, 64);
      db[c] += __shfl_xor(db[c], 32, 64);
    }
    if (lane < 16) *reinterpret_cast<float4*>(red + (wave * 16 + lane) * 4) = make_float4(db[0], db[1], db[2], db[3]);
    if (t < 5) reinterpret_cast<uint4*>(Dy + 784 * C1_DSTR)[t] = make_uint4(0, 0, 0, 0);
    bar.sync();
    if (dbg_exit == 4) return;  // profiling: conv1 tail cut after the dY1 scatter
    if (t < 64) {
      // db2 channel co4*4 + c, summed over the 32 threads with (tid & 15) == co4
      const int co4 = t >> 2, c = t & 3;
      float sacc = 0.f;
      for (int w = 0; w < 8; ++w) sacc += red[(w * 16 + co4) * 4 + c];  // 8 per-wave folds
      out_store1(cpart + (int64_t)b * CP_W + CP_DB2 + co4 * 4 + c, sacc, wt);
    } else if (t < 96) {
      // db1 channel ch = 16nt + 4lg + i
      const int ch = t - 64, nt = ch >> 4, lgg = (ch >> 2) & 3, i = ch & 3;
      float sacc = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) sacc += red1[(w * 4 + lgg) * 8 + nt * 4 + i];
      out_store1(cpart + (int64_t)b * CP_W + CP_DB1 + ch, sacc, wt);
    }
    if (dbg_exit == 5) return;  // profiling: ... after the bias sums
    // GEMM dW1^T[co][tap] = sum_pix dY1^T[co][pix] im2col(x)[pix][tap]: wave w takes image rows
    // w, w+8, w+16, w+24 (rows >= 28 read the zero dY1 row: no guard around the MFMAs).
    int boff[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = nt * 16 + lr;
      const int kh = n / 5, kw = n - (n / 5) * 5;
      boff[nt] = n < 25 ? kw * C1_XS + kh * 32 + 8 * lg : -1;
    }
    f32x4 c1[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) c1[i][0] = c1[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int y = wave + 8 * j;
      const int yb = min(y, 27);
      const int x0 = 8 * lg + q, x1 = x0 + 4;
      const int r0 = (y < 28 && x0 < 28) ? y * 28 + x0 : 784, r1 = (y < 28 && x1 < 28) ? y * 28 + x1 : 784;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        af[mt] = frag_tr(Dy + r0 * C1_DSTR + mt * 16 + 4 * p, Dy + r1 * C1_DSTR + mt * 16 + 4 * p);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) bfr[nt] = frag_ld128(boff[nt] >= 0 ? Xs + boff[nt] + yb * 32 : Zc);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) c1[mt][nt] = mfma16(af[mt], bfr[nt], c1[mt][nt]);
    }
    float* part = reinterpret_cast<float*>(D);  // [8 waves][64 lanes][16] (db areas are consumed)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        *reinterpret_cast<float4*>(part + (wave * 64 + lane) * 16 + (mt * 2 + nt) * 4) =
            make_float4(c1[mt][nt][0], c1[mt][nt][1], c1[mt][nt][2], c1[mt][nt][3]);
    bar.sync();
    if (dbg_exit == 6) return;  // profiling: ... after the GEMM (no wave sum, no stores)
    for (int o = t; o < 800; o += 512) {
      const int tap = o >> 5, co = o & 31;
      const int nt = tap >> 4, lrr = tap & 15, mt = co >> 4, lgg = (co >> 2) & 3, i = co & 3;
      const int slot = (lgg * 16 + lrr) * 16 + (mt * 2 + nt) * 4 + i;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += part[w * 64 * 16 + slot];
      out_store1(cpart + (int64_t)b * CP_W + o, v, wt);  // dW1 in HWIO order: tap * 32 + co
    }
    return;
  }
  // ======================================================================= wgrad
  const int bid = bx - n_dgrad;
  const int kh = bid % 5, grp = bid / 5;
  const int h = wave >> 2, lw = wave & 3, th = t & 255;
  u16* A = smem + h * CB_WG_GRP;   // [325][32] padded a1 image (+ zero pixel 324)
  u16* Dm = A + CB_WG_A;           // [197][64] dY2 rows = pixels (+ zero row 196)
  f32x4 acc[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ii = 0; ii < 2; ++ii) {
    const int b = grp * CB_IPB + h * 2 + ii;
    const bool active = b < B;
    const int bb = active ? b : 0;
    // loads first: a1 image chunks (interior pixels) and the dY2 items of this image
    uint4 av[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int i = min(th + 256 * k, 1299);
      const int pix = i >> 2, c = i & 3;
      const int y = pix / 18 - 2, x = pix % 18 - 2;
      const bool in = pix < 324 && y >= 0 && y < 14 && x >= 0 && x < 14;
      const int yc = in ? y : 0, xc = in ? x : 0;
      const uint4 v = *reinterpret_cast<const uint4*>(a1 + ((int64_t)bb * 196 + yc * 14 + xc) * 32 + c * 8);
      av[k] = mask_u4(v, in && active);
    }
    DyItem items[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = min(th + 256 * k, 783);
      items[k] = load_dy_item(g2, idx2, bb, (i >> 4) * 64 + (i & 15) * 4);
      // a missing image (B not a multiple of 4) contributes zeros
      const uint32_t m = active ? 0xffffffffu : 0u;
      items[k].g.x &= m;
      items[k].g.y &= m;
    }
    bar.sync();  // the previous image's operands are no longer read
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int i = th + 256 * k;
      const int pix = i >> 2, c = i & 3;
      if (i < 1300) *reinterpret_cast<uint4*>(A + pix * 32 + 8 * c) = av[k];
    }
    if (th < 8) reinterpret_cast<uint4*>(Dm + 196 * 64)[th] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = th + 256 * k;
      if (i < 784) {
        u16 g[4];
        int d[4];
        float gf[4];
        finish_dy_item(items[k], g, d, gf);
        const int win = i >> 4, grp8 = i & 15;  // 8-byte group = 4 channels
        const int py = win / 7, px = win - py * 7;
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          const int pix = (2 * py + (dd >> 1)) * 14 + 2 * px + (dd & 1);
          const uint32_t lo = (uint32_t)(d[0] == dd ? g[0] : 0) | ((uint32_t)(d[1] == dd ? g[1] : 0) << 16);
          const uint32_t hi = (uint32_t)(d[2] == dd ? g[2] : 0) | ((uint32_t)(d[3] == dd ? g[3] : 0) << 16);
          *reinterpret_cast<uint2*>(Dm + pix * 64 + 4 * (grp8 ^ swd(pix))) = make_uint2(lo, hi);
        }
      }
    }
    bar.sync();
    // (an absent image was staged as zeros, so it is computed unconditionally: no MFMA guard)
#pragma unroll
    for (int k0 = 0; k0 < 224; k0 += 32) {
      // A' = dY2^T: rows = co (16 per wave), k = pixels
      const int r0 = min(k0 + 8 * lg + q, 196), r1 = min(k0 + 8 * lg + q + 4, 196);
      const bf16x8 af = frag_tr(Dm + r0 * 64 + 4 * ((4 * lw + p) ^ swd(r0)), Dm + r1 * 64 + 4 * ((4 * lw + p) ^ swd(r1)));
      int poff[2], kwm[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int pix = k0 + 8 * lg + q + 4 * hh;
        const int y = pix / 14, x = pix - (pix / 14) * 14;
        poff[hh] = pix < 196 ? ((y + kh) * 18 + x) * 32 : 324 * 32;  // pixel 324 = zeros
        kwm[hh] = pix < 196 ? 32 : 0;
      }
#pragma unroll
      for (int mt = 0; mt < 10; ++mt) {
        const int kw = mt >> 1, ci0 = (mt & 1) * 16;
        const bf16x8 bx = frag_tr(A + poff[0] + kw * kwm[0] + ci0 + 4 * p, A + poff[1] + kw * kwm[1] + ci0 + 4 * p);
        acc[mt] = mfma16(af, bx, acc[mt]);
      }
    }
  }
  // Sum the two wave groups, then one float4 per lane per tile into the slab.
  bar.sync();
  float* red = reinterpret_cast<float*>(smem);  // group 1 -> [40][256] floats
  if (h == 1) {
#pragma unroll
    for (int mt = 0; mt < 10; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(mt * 4 + e) * 256 + th] = acc[mt][e];
  }
  bar.sync();
  if (h == 0) {
    float* out = slab + (int64_t)grp * 51200;
#pragma unroll
    for (int mt = 0; mt < 10; ++mt) {
      const int kw = mt >> 1, ci = (mt & 1) * 16 + lr;
      const int co = lw * 16 + 4 * lg;
      float4 v;
      v.x = acc[mt][0] + red[(mt * 4 + 0) * 256 + th];
      v.y = acc[mt][1] + red[(mt * 4 + 1) * 256 + th];
      v.z = acc[mt][2] + red[(mt * 4 + 2) * 256 + th];
      v.w = acc[mt][3] + red[(mt * 4 + 3) * 256 + th];
      const int oo = ((kh * 5 + kw) * 32 + ci) * 64 + co;
      if (wt) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, 51200 * 4, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(f4v{v.x, v.y, v.z, v.w}, rs, oo * 4, 0, 16);  // sc1
      } else {
        *reinterpret_cast<float4*>(out + oo) = v;
      }
    }
  }
}

// Loads of the conv roles' outputs by the reduction. SC1: the folded form (the reduction runs in
// the conv2_bwd launch after an arrival counter, cdna_hip_programming.md §6 Guideline 16): the
// producers stored them write-through (sc1), so every load of them here is an sc1 load too and no
// acquire is needed; otherwise plain loads behind the kernel boundary.
template <bool SC1>
struct ReduceLoads {
  __amdgpu_buffer_rsrc_t rs;
  const float* slab;
  const float* cpart;
  __device__ __forceinline__ ReduceLoads(const float* slab_, int nslab, const float* cpart_) : slab(slab_), cpart(cpart_) {
    if constexpr (SC1) rs = __builtin_amdgcn_make_buffer_rsrc((void*)slab_, (short)0, nslab * 51200 * 4, 0x00020000);
  }
  __device__ __forceinline__ float4 slab4(int g, int o) const {  // float4 o of slab g
    if constexpr (SC1) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rs, (g * 12800 + o) * 16, 0, 16);
      return make_float4(v[0], v[1], v[2], v[3]);
    } else {
      return reinterpret_cast<const float4*>(slab + (int64_t)g * 51200)[o];
    }
  }
  __device__ __forceinline__ float part(int64_t i) const {
    if constexpr (SC1) return __hip_atomic_load(cpart + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return cpart[i];
  }
};

// One 256-thread reduction item. Items [0, 200): dW2 = sum of the (<= 32) conv2 wgrad slabs; 64
// float4 outputs x 4 slab groups of 8 per item, every load in flight at once (absent slabs masked,
// not branched around), then a 4-way LDS sum. Items [200, 214): dW1 | db1 | db2 = sum over images
// of the per-image partial rows; 64 outputs x 4 row groups per item, 8 rows per load batch. With
// ADAM each reduced gradient is applied to its slot of the flat p/m/v/shadow buffers right away.
constexpr int CR_SLAB_BLOCKS = 200, CR_PART_BLOCKS = CP_W / 64, CR_ITEMS = CR_SLAB_BLOCKS + CR_PART_BLOCKS;
struct ReduceAdam {
  AdamArgs ad;             // p/m/v/shadow = flat buffer bases; state = the step state (read + written)
  const float* gflat;      // flat gradient buffer
  int64_t o_w2, o_w1, o_b1, o_b2;  // element offsets of the conv segments in the flat buffers
  int64_t fc_lo4, fc_hi4;  // float4 range of the fc segments updated from gflat
};
template <bool ADAM, bool SC1, class Sync>
__device__ __forceinline__ void reduce_item(int item, int t, float4* r4, Sync&& sync, const ReduceLoads<SC1>& ld,
                                            int nslab, int B, float* __restrict__ gW2, float* __restrict__ gW1,
                                            float* __restrict__ gb1, float* __restrict__ gb2, const ReduceAdam& ra,
                                            const AdamCoef& c) {
  if (item >= CR_SLAB_BLOCKS) {
    float* r1 = reinterpret_cast<float*>(r4);
    const int o = (item - CR_SLAB_BLOCKS) * 64 + (t & 63), rg = t >> 6;
    // optimizer operands first: their loads fly with the reduction's instead of after it
    int64_t f = 0;
    float pv = 0.f, mv = 0.f, vv = 0.f;
    if constexpr (ADAM) {
      if (t < 64) {
        f = o < CP_DB1 ? ra.o_w1 + o : o < CP_DB2 ? ra.o_b1 + (o - CP_DB1) : ra.o_b2 + (o - CP_DB2);
        pv = ra.ad.p[f];
        mv = ra.ad.m[f];
        vv = ra.ad.v[f];
      }
    }
    float acc = 0.f;
    for (int r0 = rg * 8; r0 < B; r0 += 32) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = r0 + k;
        v[k] = mask_f(ld.part((int64_t)min(r, B - 1) * CP_W + o), r < B);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    r1[t] = acc;
    sync();
    if (t < 64) {
      const float s = (r1[t] + r1[64 + t]) + (r1[128 + t] + r1[192 + t]);
      if (o < CP_DB1) gW1[o] = s;
      else if (o < CP_DB2) gb1[o - CP_DB1] = s;
      else gb2[o - CP_DB2] = s;
      if constexpr (ADAM) {
        adam1(pv, mv, vv, s, c);
        ra.ad.p[f] = pv;
        ra.ad.m[f] = mv;
        ra.ad.v[f] = vv;
        ra.ad.shadow[f] = f2bf(pv);
      }
    }
    return;
  }
  const int o = item * 64 + (t & 63), sg = t >> 6;  // float4 index, 12800 total
  float4 pp = make_float4(0.f, 0.f, 0.f, 0.f), mm = pp, vv = pp;
  if constexpr (ADAM) {
    if (t < 64) {  // optimizer operands in flight with the slab loads
      const int64_t f4 = ra.o_w2 / 4 + min(o, 12799);
      pp = reinterpret_cast<const float4*>(ra.ad.p)[f4];
      mm = reinterpret_cast<const float4*>(ra.ad.m)[f4];
      vv = reinterpret_cast<const float4*>(ra.ad.v)[f4];
    }
  }
  float4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int g = sg * 8 + k;
    const float4 xv = ld.slab4(min(g, nslab - 1), min(o, 12799));
    const bool keep = g < nslab;
    v[k] = make_float4(mask_f(xv.x, keep), mask_f(xv.y, keep), mask_f(xv.z, keep), mask_f(xv.w, keep));
  }
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int k = 0; k < 8; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
  r4[t] = s;
  sync();
  if (t < 64 && o < 12800) {
    const float4 a = r4[t], b = r4[64 + t], cc = r4[128 + t], d = r4[192 + t];
    const float4 g = make_float4((a.x + b.x) + (cc.x + d.x), (a.y + b.y) + (cc.y + d.y), (a.z + b.z) + (cc.z + d.z),
                                 (a.w + b.w) + (cc.w + d.w));
    reinterpret_cast<float4*>(gW2)[o] = g;
    if constexpr (ADAM) {
      const int64_t f4 = ra.o_w2 / 4 + o;
      const uint2 sh = adam4(pp, mm, vv, g, c);
      reinterpret_cast<float4*>(ra.ad.p)[f4] = pp;
      reinterpret_cast<float4*>(ra.ad.m)[f4] = mm;
      reinterpret_cast<float4*>(ra.ad.v)[f4] = vv;
      reinterpret_cast<uint2*>(ra.ad.shadow)[f4] = sh;
    }
  }
}

// Adam over the fc float4 range [fc_lo4, fc_hi4) from the gradient buffer (no conv dependency).
__device__ __forceinline__ void reduce_fc_adam(const ReduceAdam& ra, const AdamCoef& c, int64_t i, int64_t stride) {
  for (; i < ra.fc_hi4; i += stride) {
    float4 pp = reinterpret_cast<const float4*>(ra.ad.p)[i];
    const float4 gg = reinterpret_cast<const float4*>(ra.gflat)[i];
    float4 mm = reinterpret_cast<const float4*>(ra.ad.m)[i];
    float4 vv = reinterpret_cast<const float4*>(ra.ad.v)[i];
    const uint2 sh = adam4(pp, mm, vv, gg, c);
    reinterpret_cast<float4*>(ra.ad.p)[i] = pp;
    reinterpret_cast<float4*>(ra.ad.m)[i] = mm;
    reinterpret_cast<float4*>(ra.ad.v)[i] = vv;
    reinterpret_cast<uint2*>(ra.ad.shadow)[i] = sh;
  }
}

// TAIL: the launch also carries the dense/kernel Adam update — 1: from the dW3 gradient in HBM
// (AdamTail, common.h), 2: from dW3 tiles computed here from the bf16 factors (W3TileTail,
// w3_tail.h). Blocks [n_conv, grid) have no conv work and start on it at once (they sit on the CUs
// the conv roles leave idle); every conv block joins in when its own work is done.
enum { TAIL_NONE = 0, TAIL_ADAM = 1, TAIL_W3 = 2 };
// TAIL_ADAM launches may add SW streamer waves (waves 8 .. 8 + SW - 1) to every block: they stream
// the update from the first cycle on the CUs the conv roles occupy (latency-bound work that leaves
// HBM idle), while the conv waves meet on the LDS counter barrier above.
constexpr int CB_MAX_THREADS = 768;
constexpr int CB_LDS_SW = CB_LDS + 16;  // + the conv waves' barrier counter
// Folded reduction (FoldArgs, TAIL_ADAM launches with streamers): the conv2_wgrad_reduce_adam
// work runs in this launch. Every conv block stores its slab rows / partial rows write-through,
// drains them, adds 1 to an arrival counter and waits (one wave polls, bounded) for all n_conv;
// then its conv waves take reduction items (two per pass, one per 256-thread half) while the
// streamers keep streaming. The last block to pass the wait resets the counters for the next call.
struct FoldArgs {
  ReduceAdam ra;
  float *gW2, *gW1, *gb1, *gb2;
  unsigned* sync;  // [arrive, depart, error, -]: zero-initialised, reset in-kernel every call
  int nslab;
  int on;
};

// Arrival: every storing wave drains its write-through stores, then one lane counts the block in.
__device__ __forceinline__ void conv2_fold_arrive(const FoldArgs& fa, ConvBarrier<true>& bar) {
  (void)fa;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its sc1 stores have landed
  bar.sync();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add((__attribute__((address_space(1))) unsigned*)fa.sync, 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void conv2_fold_reduce(const FoldArgs& fa, ConvBarrier<true>& bar, int bx, int n_conv,
                                                  const float* slab, const float* cpart, int B) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  typedef __attribute__((address_space(1))) unsigned gu32;
  gu32* arrive = (gu32*)fa.sync;
  gu32* depart = arrive + 1;
  gu32* err = arrive + 2;
  const int t = threadIdx.x, wave = t >> 6;
  if (wave == 0) {
    // every conv block is resident (grid <= CUs, checked at launch); bounded: ~0.1 s, then an error
    int spin = 0;
    while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)n_conv) {
      if (++spin > (1 << 21)) {
        if ((t & 63) == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(16);  // ~1k cycles: up to 225 pollers share one word
    }
  }
  bar.sync();
  // every load of the handed-off slabs / partial rows below is an sc1 load: no acquire needed, only
  // keep the compiler from hoisting them above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (t == 0) {  // the whole block has passed the wait: the last one to get here resets both words
    if (__hip_atomic_fetch_add(depart, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)n_conv - 1) {
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(depart, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const ReduceAdam& ra = fa.ra;
  const AdamCoef c = adam_coef((float)ra.ad.state[ST_OPT], ra.ad.lr, ra.ad.b1, ra.ad.b2, ra.ad.eps, ra.ad.gscale,
                               ra.ad.rule);
  if (bx == 0 && t == 0) const_cast<int64_t*>(ra.ad.state)[ST_FWD] += 1;  // every conv block has read it
  const int half = t >> 8, th = t & 255;
  float4* r4 = reinterpret_cast<float4*>(smem) + half * 256;
  const ReduceLoads<true> ld(slab, fa.nslab, cpart);
  // items go to the wgrad blocks first (they finish their conv work before the dgrad blocks)
  const int n_dg = n_conv - fa.nslab * 5;
  const int rank = bx >= n_dg ? bx - n_dg : (n_conv - n_dg) + bx;
  for (int base = 2 * rank; base < CR_ITEMS; base += 2 * n_conv) {
    const int item = base + half;
    if (item < CR_ITEMS)
      reduce_item<true, true>(item, th, r4, [&] { bar.sync(); }, ld, fa.nslab, B, fa.gW2, fa.gW1, fa.gb1, fa.gb2, ra, c);
    else
      bar.sync();  // the other half's item: same barrier count
  }
  reduce_fc_adam(ra, c, ra.fc_lo4 + (int64_t)bx * 512 + t, (int64_t)n_conv * 512);
}

template <int TAIL>
__global__ void __launch_bounds__(TAIL == TAIL_ADAM ? CB_MAX_THREADS : 512) conv2_bwd_kernel(
    const u16* __restrict__ g2, const uint8_t* __restrict__ idx2,
    const u16* __restrict__ a1, const u16* __restrict__ w2bf, const float* __restrict__ x, const int* __restrict__ rows,
    int n_pool, const int64_t* __restrict__ state, const uint8_t* __restrict__ idx1, u16* __restrict__ g1,
    float* __restrict__ slab, float* __restrict__ cpart, int B, int n_dgrad, int dbg_exit, int n_conv, AdamTail at,
    W3TileTail wt, CollRole cr, FoldArgs fa) {
  // co-launched xGMI collective (xgmi_role.h) on the first cr.nblk blocks (the CUs the 225 conv
  // blocks of a B = 100 step leave idle)
  if ((int)blockIdx.x < cr.nblk) {
    coll_role_run(cr, blockIdx.x);
    return;
  }
  const int bx = (int)blockIdx.x - cr.nblk;
  if (TAIL == TAIL_ADAM && blockDim.x > 512) {
    extern __shared__ __attribute__((aligned(16))) u16 smem[];
    unsigned* ctr = reinterpret_cast<unsigned*>(smem + CB_LDS / 2);
    if (threadIdx.x == 0) *ctr = 0u;
    __syncthreads();  // the only block-wide barrier: every later one is the conv waves' own
    if (bx < n_conv && threadIdx.x < 512) {
      ConvBarrier<true> bar{ctr};
      conv2_bwd_block<true>(g2, idx2, a1, w2bf, x, rows, n_pool, state, idx1, g1, slab, cpart, B, n_dgrad, dbg_exit,
                            bx, bar, fa.on != 0);
      if constexpr (TAIL == TAIL_ADAM) {
        if (fa.on) {
          // count in, take this wave's share of the update while the other blocks finish, then reduce
          conv2_fold_arrive(fa, bar);
          adam_tail_run(at);
          conv2_fold_reduce(fa, bar, bx, n_conv, slab, cpart, B);
          return;
        }
      }
    }
  } else if (bx < n_conv) {
    ConvBarrier<false> bar{nullptr};
    conv2_bwd_block<false>(g2, idx2, a1, w2bf, x, rows, n_pool, state, idx1, g1, slab, cpart, B, n_dgrad, dbg_exit, bx,
                           bar);
  }
  if constexpr (TAIL == TAIL_ADAM) adam_tail_run(at);
  if constexpr (TAIL == TAIL_W3) w3_tail_run(wt);  // independent waves, no LDS
}

// Blocks [0, 214): one reduction item each; ADAM (world size 1): blocks [214, 214 + n_fc) update the
// fc slice, and block 0 advances the forward step — the step's last launch.
template <bool ADAM>
__global__ void __launch_bounds__(256) conv2_wgrad_reduce_kernel(const float* __restrict__ slab, int nslab,
                                                                 const float* __restrict__ cpart, int B,
                                                                 float* __restrict__ gW2, float* __restrict__ gW1,
                                                                 float* __restrict__ gb1, float* __restrict__ gb2,
                                                                 ReduceAdam ra) {
  __shared__ float4 r4[256];
  const int t = threadIdx.x;
  AdamCoef c;
  if constexpr (ADAM) {
    c = adam_coef((float)ra.ad.state[ST_OPT], ra.ad.lr, ra.ad.b1, ra.ad.b2, ra.ad.eps, ra.ad.gscale, ra.ad.rule);
    if (blockIdx.x == 0 && t == 0) const_cast<int64_t*>(ra.ad.state)[ST_FWD] += 1;
    if ((int)blockIdx.x >= CR_ITEMS) {
      reduce_fc_adam(ra, c, ra.fc_lo4 + ((int64_t)blockIdx.x - CR_ITEMS) * 256 + t,
                     (int64_t)(gridDim.x - CR_ITEMS) * 256);
      return;
    }
  }
  const ReduceLoads<false> ld(slab, nslab, cpart);
  reduce_item<ADAM, false>((int)blockIdx.x, t, r4, [] { __syncthreads(); }, ld, nslab, B, gW2, gW1, gb1, gb2, ra, c);
}

// ------------------------------------------------------------------------------------------ //
int64_t conv2_wgrad_groups(int64_t B) { return (B + CB_IPB - 1) / CB_IPB; }
static int64_t B_of(const at::Tensor& a1) { return a1.size(0); }

static void conv2_bwd_launch(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                             const at::Tensor& x, const c10::optional<at::Tensor>& rows,
                             const c10::optional<at::Tensor>& state, const at::Tensor& idx1, at::Tensor& slab,
                             at::Tensor& cpart, const c10::optional<at::Tensor>& g1, const AdamTail* tail,
                             int64_t coll, const W3TileTail* w3t = nullptr, const FoldArgs* fold = nullptr,
                             bool* fold_done = nullptr) {
  const int B = a1.size(0);
  const int G = (int)conv2_wgrad_groups(B);
  TORCH_CHECK(g2.dtype() == MIHVD_OP16 && g2.numel() == (int64_t)B * 3136 && idx2.numel() == g2.numel(), "conv2_bwd: g2/idx2");
  TORCH_CHECK(a1.dtype() == MIHVD_OP16 && a1.numel() == (int64_t)B * 6272 && idx1.numel() == a1.numel() &&
                  idx1.dtype() == at::kByte, "conv2_bwd: a1/idx1");
  TORCH_CHECK(w2bf.dtype() == MIHVD_OP16 && w2bf.numel() == 51200, "conv2_bwd: w2");
  TORCH_CHECK(x.dtype() == at::kFloat && x.size(-1) == 784 && x.is_contiguous(), "conv2_bwd: x");
  TORCH_CHECK(slab.dtype() == at::kFloat && slab.numel() >= (int64_t)G * 51200, "conv2_bwd: slab must hold ceil(B/4) x 51200");
  TORCH_CHECK(cpart.dtype() == at::kFloat && cpart.numel() >= (int64_t)B * CP_W && cpart.is_contiguous(),
              "conv2_bwd: cpart must hold B x 896 floats (per-image dW1 | db1 | db2)");
  u16* g1p = nullptr;
  if (g1.has_value() && g1->defined()) {
    TORCH_CHECK(g1->dtype() == MIHVD_OP16 && g1->numel() == a1.numel(), "conv2_bwd: g1");
    g1p = (u16*)g1->data_ptr();
  }
  const int* rp = nullptr;
  int n_pool = x.size(0);
  if (rows.has_value() && rows->defined()) rp = rows->data_ptr<int>();
  else TORCH_CHECK(n_pool >= B, "conv2_bwd: x has fewer rows than the batch");
  const int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  static bool attr = [] {
    for (const void* f : {(const void*)conv2_bwd_kernel<TAIL_NONE>, (const void*)conv2_bwd_kernel<TAIL_ADAM>,
                          (const void*)conv2_bwd_kernel<TAIL_W3>}) {
      hipFuncAttributes fa;
      TORCH_CHECK(hipFuncGetAttributes(&fa, f) == hipSuccess, "conv2_bwd: hipFuncGetAttributes");
      TORCH_CHECK(fa.sharedSizeBytes + CB_LDS_SW <= 163840, "conv2_bwd: static (", fa.sharedSizeBytes, ") + dynamic (",
                  CB_LDS_SW, ") LDS exceeds the CU's 163,840 B");
      TORCH_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, CB_LDS_SW) == hipSuccess,
                  "conv2_bwd: hipFuncSetAttribute");
    }
    return true;
  }();
  (void)attr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  const int role = debug_role_only();  // 0: dgrad blocks only, 1: wgrad blocks only, 2: no conv blocks
  const int n_dgrad = role == 1 ? 0 : B;
  const int n_conv = role == 2 ? 0 : role == 0 ? B : role == 1 ? 5 * G : B + 5 * G;
  const CollRole cr = xgmi_role_lookup(coll);
  if (w3t != nullptr) {
    // one 512-thread block per CU (144 KB of LDS): the tail-only blocks take the CUs the conv roles
    // leave free and start on the dW3 tiles at once (their share of the tiles tuned on MI355X)
    const int ncu = device_cu_count();
    const int grid = std::max(n_conv + 8, ncu);
    constexpr double head_frac = 0.25;
    W3TileTail wtl = *w3t;
    wtl.first_free = n_conv;
    wtl.head = (int)(head_frac * W3T_TILES);
    if (role == 2) wtl.first_free = 0;  // kbench: the tail alone
    TORCH_CHECK(cr.nblk == 0, "conv2_bwd_w3adam: no co-launched collective with the optimizer tail");
    conv2_bwd_kernel<TAIL_W3><<<grid, 512, CB_LDS, stream>>>(
        (const u16*)g2.data_ptr(), idx2.data_ptr<uint8_t>(), (const u16*)a1.data_ptr(), (const u16*)w2bf.data_ptr(),
        x.data_ptr<float>(), rp, n_pool, sp, idx1.data_ptr<uint8_t>(), g1p, slab.data_ptr<float>(),
        cpart.data_ptr<float>(), B, n_dgrad, debug_phase_exit(), n_conv, AdamTail{}, wtl, cr, FoldArgs{});
  } else if (tail == nullptr) {
    conv2_bwd_kernel<TAIL_NONE><<<cr.nblk + n_conv, 512, CB_LDS, stream>>>(
        (const u16*)g2.data_ptr(), idx2.data_ptr<uint8_t>(), (const u16*)a1.data_ptr(), (const u16*)w2bf.data_ptr(),
        x.data_ptr<float>(), rp, n_pool, sp, idx1.data_ptr<uint8_t>(), g1p, slab.data_ptr<float>(),
        cpart.data_ptr<float>(), B, n_dgrad, debug_phase_exit(), n_conv, AdamTail{}, W3TileTail{}, cr, FoldArgs{});
  } else {
    // one block per CU (the conv roles' LDS): the extra tail-only blocks take the CUs the conv
    // roles leave free, and every conv block carries streamer waves, so the update streams from
    // the first cycle on every CU (the conv roles are latency-bound and leave HBM idle)
    const int ncu = device_cu_count();
    const int grid = std::max(n_conv + 8, ncu);
    // four streamer waves per compute block (768 threads)
    constexpr int sw = 4;
    const int nthr = debug_phase_exit() ? 512 : 512 + 64 * sw;  // profiling cuts: conv waves alone
    // The free waves' head range (their fraction of the update), tuned on MI355X: with streamers
    // they carry most of the update while the conv roles run.
    constexpr double head_frac = 0.8;
    AdamTail at = *tail;
    at.first_free = n_conv;
    at.head = (int64_t)(head_frac * (double)((at.n4 + 63) / 64));
    TORCH_CHECK(cr.nblk == 0, "conv2_bwd_adam: no co-launched collective with the optimizer tail");
    // The folded reduction needs every conv block resident at once (they wait for each other) and
    // the streamer form (its barrier); otherwise the caller's separate reduce launch runs.
    FoldArgs fa = fold ? *fold : FoldArgs{};
    fa.on = fold != nullptr && nthr > 512 && role == -1 && n_conv <= grid && grid <= ncu;
    if (fold) *fold_done = fa.on != 0;
    conv2_bwd_kernel<TAIL_ADAM><<<grid, nthr, nthr > 512 ? CB_LDS_SW : CB_LDS, stream>>>(
        (const u16*)g2.data_ptr(), idx2.data_ptr<uint8_t>(), (const u16*)a1.data_ptr(), (const u16*)w2bf.data_ptr(),
        x.data_ptr<float>(), rp, n_pool, sp, idx1.data_ptr<uint8_t>(), g1p, slab.data_ptr<float>(),
        cpart.data_ptr<float>(), B, n_dgrad, debug_phase_exit(), n_conv, at, W3TileTail{}, cr, fa);
  }
}

void conv2_bwd(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
               const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, const c10::optional<at::Tensor>& g1,
               int64_t coll) {
  conv2_bwd_launch(g2, idx2, a1, w2bf, x, rows, state, idx1, slab, cpart, g1, nullptr, coll);
}

static void check_flat(const at::Tensor& t, at::ScalarType dt, int64_t n, const char* what) {
  TORCH_CHECK(t.scalar_type() == dt && t.numel() == n && t.is_contiguous() && ((uintptr_t)t.data_ptr() & 15) == 0, what);
}

// conv2_bwd + the Adam update of a flat slice (p3/g3/m3/v3/shadow3: the dense/kernel segment) in
// the launch's tail (AdamTail, common.h).
void conv2_bwd_adam(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                    const at::Tensor& x, const c10::optional<at::Tensor>& rows, at::Tensor& state, const at::Tensor& idx1,
                    at::Tensor& slab, at::Tensor& cpart, at::Tensor& p3, const at::Tensor& g3, at::Tensor& m3,
                    at::Tensor& v3, at::Tensor& shadow3, double lr, double b1, double b2, double eps, double grad_scale,
                    int64_t rule) {
  const int64_t n = p3.numel();
  TORCH_CHECK(n % 4 == 0 && n > 0, "conv2_bwd_adam: slice length must be a positive multiple of 4");
  check_flat(p3, at::kFloat, n, "conv2_bwd_adam: p3");
  check_flat(g3, at::kFloat, n, "conv2_bwd_adam: g3");
  check_flat(m3, at::kFloat, n, "conv2_bwd_adam: m3");
  check_flat(v3, at::kFloat, n, "conv2_bwd_adam: v3");
  check_flat(shadow3, MIHVD_OP16, n, "conv2_bwd_adam: shadow3");
  TORCH_CHECK(state.scalar_type() == at::kLong && state.numel() >= ST_WORDS, "conv2_bwd_adam: state");
  AdamTail at{p3.data_ptr<float>(), g3.data_ptr<float>(), m3.data_ptr<float>(), v3.data_ptr<float>(),
              (u16*)shadow3.data_ptr(), n / 4, state.data_ptr<int64_t>(), (float)lr, (float)b1, (float)b2,
              (float)eps, (float)grad_scale, (int)rule, 0, 0};
  conv2_bwd_launch(g2, idx2, a1, w2bf, x, rows, state, idx1, slab, cpart, c10::nullopt, &at, -1);
}

// conv2_bwd + the dense/kernel Adam update from dW3 = a2^T dz tiles computed in the launch's tail
// (W3TileTail, w3_tail.h): dzT [1024][128] and a2T [3136][128] bf16 are this step's fc1 factors,
// transposed by fc1_bwd's dgrad blocks (zero past the batch); p3/m3/v3/shadow3 the dense/kernel
// segments of the flat buffers; gW3 (optional) also receives dW3.
void conv2_bwd_w3adam(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                      const at::Tensor& x, const c10::optional<at::Tensor>& rows, at::Tensor& state,
                      const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, const at::Tensor& dzT,
                      const at::Tensor& a2T, at::Tensor& p3, at::Tensor& m3, at::Tensor& v3, at::Tensor& shadow3,
                      const c10::optional<at::Tensor>& gW3, double lr, double b1, double b2, double eps,
                      double grad_scale, int64_t rule) {
  const int B = a1.size(0);
  const int64_t n = (int64_t)W3T_K * W3T_N;
  TORCH_CHECK(B >= 1 && B <= W3T_KP, "conv2_bwd_w3adam: batch must be in [1, 128]");
  check_flat(dzT, MIHVD_OP16, (int64_t)W3T_N * W3T_KP, "conv2_bwd_w3adam: dzT [1024][128] bf16");
  check_flat(a2T, MIHVD_OP16, (int64_t)W3T_K * W3T_KP, "conv2_bwd_w3adam: a2T [3136][128] bf16");
  check_flat(p3, at::kFloat, n, "conv2_bwd_w3adam: p3");
  check_flat(m3, at::kFloat, n, "conv2_bwd_w3adam: m3");
  check_flat(v3, at::kFloat, n, "conv2_bwd_w3adam: v3");
  check_flat(shadow3, MIHVD_OP16, n, "conv2_bwd_w3adam: shadow3");
  float* gp = nullptr;
  if (gW3.has_value() && gW3->defined()) {
    check_flat(*gW3, at::kFloat, n, "conv2_bwd_w3adam: gW3");
    gp = gW3->data_ptr<float>();
  }
  TORCH_CHECK(state.scalar_type() == at::kLong && state.numel() >= ST_WORDS, "conv2_bwd_w3adam: state");
  W3TileTail wt{(const u16*)dzT.data_ptr(), (const u16*)a2T.data_ptr(),
                AdamArgs{p3.data_ptr<float>(), m3.data_ptr<float>(), v3.data_ptr<float>(), (u16*)shadow3.data_ptr(),
                         state.data_ptr<int64_t>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale,
                         (int)rule},
                gp, 0, 0};
  conv2_bwd_launch(g2, idx2, a1, w2bf, x, rows, state, idx1, slab, cpart, c10::nullopt, nullptr, -1, &wt);
}

void conv2_wgrad_reduce(const at::Tensor& slab, const at::Tensor& cpart, int64_t B, at::Tensor& gW2, at::Tensor& gW1,
                        at::Tensor& gb1, at::Tensor& gb2) {
  const int G = (int)conv2_wgrad_groups(B);
  TORCH_CHECK(G >= 1 && G <= 32, "conv2_wgrad_reduce: at most 32 wgrad slabs");
  TORCH_CHECK(slab.dtype() == at::kFloat && slab.numel() >= (int64_t)G * 51200, "conv2_wgrad_reduce: slab");
  TORCH_CHECK(cpart.dtype() == at::kFloat && cpart.numel() >= B * CP_W, "conv2_wgrad_reduce: cpart");
  TORCH_CHECK(gW2.dtype() == at::kFloat && gW2.numel() == 51200 && gW2.is_contiguous(), "conv2_wgrad_reduce: gW2");
  TORCH_CHECK(gW1.numel() == 800 && gb1.numel() == 32 && gb2.numel() == 64 && gW1.dtype() == at::kFloat &&
                  gb1.dtype() == at::kFloat && gb2.dtype() == at::kFloat, "conv2_wgrad_reduce: gW1/gb1/gb2");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  conv2_wgrad_reduce_kernel<false><<<CR_SLAB_BLOCKS + CR_PART_BLOCKS, 256, 0, stream>>>(
      slab.data_ptr<float>(), G, cpart.data_ptr<float>(), (int)B, gW2.data_ptr<float>(), gW1.data_ptr<float>(),
      gb1.data_ptr<float>(), gb2.data_ptr<float>(), ReduceAdam{});
}

// conv2_wgrad_reduce + Adam for every parameter outside [w3_lo, end) of the flat buffers: the conv
// gradients straight from the reduction, [fc_lo, w3_lo) from the gradient buffer. gW2/gW1/gb1/gb2
// must be views of `grads` (their offsets locate the parameters). Advances state[ST_FWD]: the
// last launch of a world-size-1 step.
static ReduceAdam make_reduce_adam(const at::Tensor& slab, const at::Tensor& cpart, int64_t B, at::Tensor& gW2,
                                   at::Tensor& gW1, at::Tensor& gb1, at::Tensor& gb2, const at::Tensor& grads,
                                   at::Tensor& p, at::Tensor& m, at::Tensor& v, at::Tensor& shadow, at::Tensor& state,
                                   int64_t fc_lo, int64_t w3_lo, double lr, double b1, double b2, double eps,
                                   double grad_scale, int64_t rule) {
  const int G = (int)conv2_wgrad_groups(B);
  TORCH_CHECK(G >= 1 && G <= 32, "conv2_wgrad_reduce_adam: at most 32 wgrad slabs");
  TORCH_CHECK(slab.dtype() == at::kFloat && slab.numel() >= (int64_t)G * 51200, "conv2_wgrad_reduce_adam: slab");
  TORCH_CHECK(cpart.dtype() == at::kFloat && cpart.numel() >= B * CP_W, "conv2_wgrad_reduce_adam: cpart");
  const int64_t n = grads.numel();
  check_flat(grads, at::kFloat, n, "conv2_wgrad_reduce_adam: grads");
  check_flat(p, at::kFloat, n, "conv2_wgrad_reduce_adam: p");
  check_flat(m, at::kFloat, n, "conv2_wgrad_reduce_adam: m");
  check_flat(v, at::kFloat, n, "conv2_wgrad_reduce_adam: v");
  check_flat(shadow, MIHVD_OP16, n, "conv2_wgrad_reduce_adam: shadow");
  TORCH_CHECK(state.scalar_type() == at::kLong && state.numel() >= ST_WORDS, "conv2_wgrad_reduce_adam: state");
  TORCH_CHECK(fc_lo % 4 == 0 && w3_lo % 4 == 0 && 0 <= fc_lo && fc_lo <= w3_lo && w3_lo <= n,
              "conv2_wgrad_reduce_adam: fc_lo/w3_lo");
  const float* g0 = grads.data_ptr<float>();
  auto off = [&](const at::Tensor& t, int64_t len, const char* what) {
    TORCH_CHECK(t.dtype() == at::kFloat && t.numel() == len && t.is_contiguous(), what);
    const int64_t o = t.data_ptr<float>() - g0;
    TORCH_CHECK(o >= 0 && o + len <= fc_lo, what, " must be a view of grads below fc_lo");
    return o;
  };
  ReduceAdam ra;
  ra.ad = AdamArgs{p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), (u16*)shadow.data_ptr(),
                   state.data_ptr<int64_t>(), (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale, (int)rule};
  ra.gflat = g0;
  ra.o_w2 = off(gW2, 51200, "conv2_wgrad_reduce_adam: gW2");
  TORCH_CHECK(ra.o_w2 % 4 == 0, "conv2_wgrad_reduce_adam: gW2 must be 16-byte aligned");
  ra.o_w1 = off(gW1, 800, "conv2_wgrad_reduce_adam: gW1");
  ra.o_b1 = off(gb1, 32, "conv2_wgrad_reduce_adam: gb1");
  ra.o_b2 = off(gb2, 64, "conv2_wgrad_reduce_adam: gb2");
  ra.fc_lo4 = fc_lo / 4;
  ra.fc_hi4 = w3_lo / 4;
  return ra;
}

static void launch_reduce_adam(const ReduceAdam& ra, const at::Tensor& slab, const at::Tensor& cpart, int64_t B,
                               at::Tensor& gW2, at::Tensor& gW1, at::Tensor& gb1, at::Tensor& gb2) {
  const int G = (int)conv2_wgrad_groups(B);
  // the fc range may include part of dense/kernel (the trainer's split): up to 4 blocks per CU
  const int n_fc = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (ra.fc_hi4 - ra.fc_lo4 + 255) / 256));
  auto stream = c10::hip::getCurrentHIPStream().stream();
  conv2_wgrad_reduce_kernel<true><<<CR_SLAB_BLOCKS + CR_PART_BLOCKS + n_fc, 256, 0, stream>>>(
      slab.data_ptr<float>(), G, cpart.data_ptr<float>(), (int)B, gW2.data_ptr<float>(), gW1.data_ptr<float>(),
      gb1.data_ptr<float>(), gb2.data_ptr<float>(), ra);
}

void conv2_wgrad_reduce_adam(const at::Tensor& slab, const at::Tensor& cpart, int64_t B, at::Tensor& gW2,
                             at::Tensor& gW1, at::Tensor& gb1, at::Tensor& gb2, const at::Tensor& grads, at::Tensor& p,
                             at::Tensor& m, at::Tensor& v, at::Tensor& shadow, at::Tensor& state, int64_t fc_lo,
                             int64_t w3_lo, double lr, double b1, double b2, double eps, double grad_scale,
                             int64_t rule) {
  const ReduceAdam ra = make_reduce_adam(slab, cpart, B, gW2, gW1, gb1, gb2, grads, p, m, v, shadow, state, fc_lo, w3_lo,
                                         lr, b1, b2, eps, grad_scale, rule);
  launch_reduce_adam(ra, slab, cpart, B, gW2, gW1, gb1, gb2);
}

// conv2_bwd_adam + conv2_wgrad_reduce_adam as ONE launch when the folded reduction applies
// (FoldArgs: streamer form, every conv block resident); otherwise the same two launches. The
// dense/kernel update covers [w3_lo, end) of the flat buffers; sync: int32 [4] zeros, owned by the
// caller (reset in-kernel after every call; word 2 = 1 after a timed-out wait).
void conv2_bwd_adam_fold(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf,
                         const at::Tensor& x, const c10::optional<at::Tensor>& rows, at::Tensor& state,
                         const at::Tensor& idx1, at::Tensor& slab, at::Tensor& cpart, at::Tensor& gW2, at::Tensor& gW1,
                         at::Tensor& gb1, at::Tensor& gb2, const at::Tensor& grads, at::Tensor& p, at::Tensor& m,
                         at::Tensor& v, at::Tensor& shadow, at::Tensor& sync, int64_t fc_lo, int64_t w3_lo, double lr,
                         double b1, double b2, double eps, double grad_scale, int64_t rule) {
  const ReduceAdam ra = make_reduce_adam(slab, cpart, B_of(a1), gW2, gW1, gb1, gb2, grads, p, m, v, shadow, state, fc_lo,
                                         w3_lo, lr, b1, b2, eps, grad_scale, rule);
  const int64_t n = grads.numel();
  TORCH_CHECK(n - w3_lo > 0 && (n - w3_lo) % 4 == 0, "conv2_bwd_adam_fold: dense/kernel slice");
  TORCH_CHECK(sync.scalar_type() == at::kInt && sync.numel() >= 4 && sync.is_contiguous(), "conv2_bwd_adam_fold: sync");
  AdamTail at{p.data_ptr<float>() + w3_lo, grads.data_ptr<float>() + w3_lo, m.data_ptr<float>() + w3_lo,
              v.data_ptr<float>() + w3_lo, (u16*)shadow.data_ptr() + w3_lo, (n - w3_lo) / 4, state.data_ptr<int64_t>(),
              (float)lr, (float)b1, (float)b2, (float)eps, (float)grad_scale, (int)rule, 0, 0};
  FoldArgs fa{ra, gW2.data_ptr<float>(), gW1.data_ptr<float>(), gb1.data_ptr<float>(), gb2.data_ptr<float>(),
              (unsigned*)sync.data_ptr<int>(), (int)conv2_wgrad_groups(B_of(a1)), 1};
  bool done = false;
  conv2_bwd_launch(g2, idx2, a1, w2bf, x, rows, state, idx1, slab, cpart, c10::nullopt, &at, -1, nullptr, &fa, &done);
  if (!done) launch_reduce_adam(ra, slab, cpart, B_of(a1), gW2, gW1, gb1, gb2);
}

MIHVD_OPNS_END

#ifndef MIHVD_F16
namespace mihvd {
// Read (and with reset, clear) the conv barrier error word; waits for the current stream.
int64_t conv_barrier_error(bool reset) {
  auto stream = c10::hip::getCurrentHIPStream().stream();
  unsigned v = 0;
  TORCH_CHECK(hipStreamSynchronize(stream) == hipSuccess, "conv_barrier_error: stream sync failed");
  TORCH_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_conv_barrier_err), sizeof(v)) == hipSuccess,
              "conv_barrier_error: read failed");
  if (reset && v) {
    const unsigned z = 0;
    TORCH_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_conv_barrier_err), &z, sizeof(z)) == hipSuccess,
                "conv_barrier_error: reset failed");
  }
  return (int64_t)v;
}
}  // namespace mihvd
#endif
