// Exact-fp32 forward kernels of the MNIST CNN (horovod/tensorflow_mnist.py:38-73).
//
// The reference's launched entrypoint trains in fp32 — fp32 placeholders (:118-121) and
// AdamOptimizer (:130) on fp32 variables — so this step keeps every operand fp32. GEMM-shaped work
// runs on the fp32-input matrix cores: v_mfma_f32_16x16x4_f32 (one fp32 A and B value per lane,
// exact products, fp32 accumulation; gfx950 has no reduced-precision xf32 form). Activations,
// gradients, weights and optimizer state are fp32 throughout.
//
// Operand convention (f32_common.h): both operands of a 16x16x4 MFMA are read as float4 chunks of
// 4 consecutive k per lane where the tensor is K-contiguous; lane group g (= lane >> 4) holds
// k = 4g + j in element j, and the four MFMAs of the chunk use elements j = 0..3. The same k order
// on both operands makes the chunk's 16-deep dot product exact (only the fp32 summation order
// differs from a sequential loop).
//
//   f32_conv1_fwd  conv1 (K = 25 taps in 7 MFMAs, x in LDS) + bias + ReLU + 2x2 pool/argmax
//   f32_conv2_fwd  conv2 over 16-pixel tiles of the whole batch (pool-window-major rows), ~one
//                  block per CU; a1 rows staged once in LDS, W2 fragments from L2 two taps ahead
//   f32_fc1_fwd    split-K (14 slices of 224) partial slabs; W3 fragments held in registers
//   f32_head       slab sum + bias + ReLU + dropout + fc2 + softmax-xent + fc2 backward -> dz
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "f32_common.h"

namespace mihvd {

// Phase stamps of f32_conv2_fwd blocks (study instrument; f32_stamps_enable(1, n) in f32_bwd.hip
// sets the buffer): slots 0 start, 1 staging barrier, 2 + pair index: end of each tile pair.
// (compiled in only by a study build, MIHVD_F32_STAMPS: see c2b_stamp in f32_bwd.hip)
__device__ unsigned long long* g_c2f_stamps = nullptr;
__device__ __forceinline__ void c2f_stamp(int k) {
#ifdef MIHVD_F32_STAMPS
  unsigned long long* p = g_c2f_stamps;
  if (p != nullptr && threadIdx.x == 0) p[blockIdx.x * 16 + k] = __builtin_amdgcn_s_memtime();
#endif
}
void f32_fwd_stamps_set(unsigned long long* p) {
  TORCH_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_c2f_stamps), &p, sizeof(p)) == hipSuccess, "c2f stamps");
}

// ------------------------------------------------------------------------------------------ //
// conv1: x rows [784] fp32 -> a1 [B][14][14][32] fp32 + argmax idx1 (u8)
// grid (4, B): block q of an image owns the 16-row tiles [13q, 13q + 13) of its 49 (4 pooling
// windows per tile, pool-window-major: row m = 4 * window + d, d = 2 * dy + dx). 4 waves, wave w:
// tiles 13q + w, +4, ... . A = im2col(x) gathered from the padded image in LDS (one ds_read_b32
// per MFMA), B = W1 in registers (k = 4s + lane group, 25 taps zero-padded to 28).
// ------------------------------------------------------------------------------------------ //
// W2 fragment copies (MIHVD_F32_W2F): the register-resident W2 operands of conv2_fwd and of the
// conv2_bwd dgrad blocks, each stored in the order the waves load them, so every load instruction
// of a wave reads one contiguous 1 KB (a float4 per lane) instead of 16 (or 4) scattered 64-byte
// pieces of the HWIO tensor: fewer load instructions (conv2_fwd: 50 instead of 200 per lane) and
// whole 128-byte lines through the CU's L1. Written from W2 by extra blocks of the conv1 launch,
// which precedes both readers in every step (W2 changes only in the step's final Adam).
//   fwd [tap][c2][wave 4][lane][j] = W2[tap][16 c2 + 4 lg + j][16 wave + lr]
//   bwd [wave 8][tap][lane][j]     = W2[tap][16 (wave & 1) + lr][16 (wave >> 1) + 4 lg + j]
constexpr int W2F_F4 = 12800;                     // float4 per copy
constexpr int W2F_BLOCKS_Y = 7;                   // extra grid rows of the conv1 launch (4 x 7 blocks)
__device__ __forceinline__ void f32_w2_frag_block(int blk, const float* __restrict__ w2, float* __restrict__ w2f) {
  float4* out = reinterpret_cast<float4*>(w2f);
  for (int i = blk * 256 + (int)threadIdx.x; i < 2 * W2F_F4; i += 4 * W2F_BLOCKS_Y * 256) {
    float4 v;
    if (i < W2F_F4) {
      const int lane = i & 63, wave = (i >> 6) & 3, c2 = (i >> 8) & 1, tap = i >> 9;
      const float* q = w2 + tap * 2048 + (16 * c2 + 4 * (lane >> 4)) * 64 + 16 * wave + (lane & 15);
      v = make_float4(q[0], q[64], q[128], q[192]);
    } else {
      const int k = i - W2F_F4, lane = k & 63, tap = (k >> 6) % 25, wave = (k >> 6) / 25;
      v = *reinterpret_cast<const float4*>(w2 + tap * 2048 + (16 * (wave & 1) + (lane & 15)) * 64 +
                                           16 * (wave >> 1) + 4 * (lane >> 4));
    }
    out[i] = v;
  }
}

__global__ void __launch_bounds__(256) f32_conv1_kernel(
    const float* __restrict__ x, const int* __restrict__ rows, int n_pool, const int64_t* __restrict__ state,
    const float* __restrict__ w1, const float* __restrict__ b1, float* __restrict__ a1, uint8_t* __restrict__ idx1,
    int B, const float* __restrict__ w2, float* __restrict__ w2f) {
  __shared__ float xim[32 * 32];  // 28 x 28 image with a 2-pixel zero halo
  const int id = blockIdx.x;
  if (id >= 4 * B) {
    f32_w2_frag_block(id - 4 * B, w2, w2f);
    return;
  }
  // XCD-contiguous (image, quarter) order: XCD x writes the a1 rows of images [B x / 8, B (x + 1) / 8),
  // the images whose conv2_fwd blocks run on XCD x (same mapping there), so conv2_fwd's staging
  // reads hit that XCD's L2 instead of the MALL
  const int L = xcd_contiguous(id, 0, 4 * B);
  f32_conv1_block<false>(L & 3, L >> 2, x, rows, n_pool, state, w1, b1, a1, idx1, B, xim);
}

// ------------------------------------------------------------------------------------------ //
// conv2: a1 [B][14][14][32] -> a2 [B][3136] (NHWC flatten of [7][7][64]) + idx2
//
// M = the 49 B pooling windows of the batch x 4 pixels (pool-window-major), in 16-row tiles; block
// b owns tiles [b TPB, (b+1) TPB) (TPB = ceil(tiles / 256): about one block per CU), which span at
// most two images. The a1 rows those tiles read are staged once as rows of the "tall" padded image
// (image i = tall rows [18 i, 18 i + 18), padded row r = a1 row r - 2, 18 padded columns of a
// 24-pixel row, pixel stride 36 floats). 4 waves, one per SIMD; wave w owns output channels
// 16w..16w+15.
//
// Weights stay in registers: a wave's whole B operand (W2[tap][ci][16w..16w+15], 800 k x 16 co =
// 200 floats per lane) is loaded once, so the MFMA loop has no global load and no barrier; only
// the A chunks come from LDS (one ds_read_b128 per 4 MFMAs, shared by the 4 waves). Tiles are
// processed in pairs with alternating accumulators (16x16x4 f32: 32-cycle issue, 40-cycle
// dependent latency), the 25 taps fully unrolled (constant LDS offsets, static register indices).
// Epilogue: 2x2 max-pool + argmax + bias + ReLU in registers.
// ------------------------------------------------------------------------------------------ //
// Pixel stride 40 floats, 20 pixels per tall row (18 used). A ds_read_b128 is serviced in four
// 16-lane groups, each pairing the lanes of two 4-channel chunks (lane groups lg 0/1 or 2/3) of 8
// pixel rows each, over every tap offset and every window-row wrap of a tile; this stride and row
// length give 1.4 LDS cycles per group on average (scripts/ldssim_conv2.py: exhaustive over the
// B = 100 tiles and taps), against 2.3 for the 36 x 24 layout before (PMC: LDS_BANK_CONFLICT 3.5x
// the active LDS cycles) and 1.0 only for tile shapes that leave MFMA rows idle.
constexpr int C2F_PS = 40, C2F_RW = 20, C2F_RS = C2F_RW * C2F_PS, C2F_MAXR = 22;
constexpr int C2F_LDS = C2F_MAXR * C2F_RS * 4;                     // 70,400 B
constexpr int C2F_MAXCH = (C2F_MAXR * 18 * 8 + 255) / 256;         // image float4 chunks per thread

// A row (tall-image offset) of lane row lr of tile `tile` (clamped past the batch)
__device__ __forceinline__ int c2f_abase(int tile, int lr, int lg, int nwin, int R0) {
  const int m = 16 * tile + lr;
  const int gw = min(m >> 2, nwin - 1), d = m & 3;
  const int bb = gw / 49, win = gw - 49 * bb, py = win / 7, px = win - 7 * py;
  const int y = 2 * py + (d >> 1), xx = 2 * px + (d & 1);
  return ((18 * bb + y - R0) * C2F_RW + xx) * C2F_PS + 4 * lg;
}

// NT (1 or 2) tiles against the register-resident weights: acc[u] += A(tile u) x W2. Software
// pipeline over the 50 (tap, 16-channel) steps, fully unrolled: the A chunks of step s + 1 are read
// into the other register set before step s's MFMAs issue (sched_barrier pins the order).
// DEPTH: steps the A reads run ahead of the MFMAs (1, or 2 with a third register set; one wave per
// SIMD has no other wave to cover an LDS latency the prefetch leaves exposed).
template <int NT, int DEPTH = 2>
__device__ __forceinline__ void c2f_tiles(const float* img, const int (&ab)[2], const float (&wb)[200],
                                          f32x4 (&acc)[2]) {
  constexpr int R = DEPTH + 1;
  float4 ra[R][NT];
  auto load_a = [&](float4 (&a)[NT], int st) {
    const int tap = st >> 1, c2 = st & 1, kh = tap / 5, kw = tap - 5 * kh;
    const int off = (kh * C2F_RW + kw) * C2F_PS + 16 * c2;
#pragma unroll
    for (int u = 0; u < NT; ++u) a[u] = *reinterpret_cast<const float4*>(img + ab[u] + off);
  };
  auto mfma_step = [&](const float4 (&a)[NT], int st) {
    const float* w = wb + 4 * st;  // wb[8 tap + 4 c2 + j]
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].x, w[0], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].y, w[1], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].z, w[2], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].w, w[3], acc[u]);
  };
#pragma unroll
  for (int st = 0; st < DEPTH; ++st) load_a(ra[st], st);
#pragma unroll
  for (int st = 0; st < 50; ++st) {
    if (st + DEPTH < 50) load_a(ra[(st + DEPTH) % R], st + DEPTH);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(ra[st % R], st);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// TAIL: the first ad.nblk blocks of the launch stream an Adam update instead (the previous step's
// dense/kernel update, deferred into this MFMA-bound launch, which leaves HBM idle). They are first
// in dispatch order, so they take the CUs before the conv blocks; a tail block and a conv block fit
// one CU together when registers allow (2 x 76 KB of LDS).
// A block barrier that orders LDS only (see lds_barrier in f32_bwd.hip): the W2 register prefetch
// stays in flight across it.
__device__ __forceinline__ void c2f_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// conv1 operands of the fused conv1 + conv2 forward (FUSE1): the block computes the a1 rows its
// conv2 tiles read (their halo included) straight from x, instead of loading them from a1.
struct C1Fuse {
  const float* x = nullptr;
  const int* rows = nullptr;
  int n_pool = 0;
  const int64_t* state = nullptr;
  const float* w1 = nullptr;
  const float* b1 = nullptr;
  float* a1 = nullptr;     // written for the backward: the rows of the block's own window rows
  uint8_t* idx1 = nullptr;
};
constexpr int C2F_XIM = 2 * 1024;  // two padded x images [32][32] after the tall image

// FUSE1 staging: conv1 (25 taps on 16x16x4 MFMA, as f32_conv1_block) of the a1 rows in tall rows
// [R0, R1) of images b0 .. b1i, pooled + bias + ReLU straight into the tall padded LDS image (whose
// padding was zeroed), and into a1 / idx1 for the rows of this block's own conv2 window rows (rows
// two blocks share are written by both, with identical values).
__device__ __forceinline__ void c2f_conv1_stage(const C1Fuse& c1, float* img, float* xim, int B, int R0, int R1,
                                                int b0, int b1i, int gw0, int gw1) {
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  float wb1[2][7];
  int toff[7];
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    const int k = 4 * s + lg, kc = min(k, 24);
    toff[s] = (kc / 5) * 32 + (kc % 5);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) wb1[nt][s] = mask_f(c1.w1[kc * 32 + 16 * nt + lr], k < 25);
  }
  const float bias0 = c1.b1[lr], bias1 = c1.b1[16 + lr];
  // window segments (a1 pixels) of the two images, in tiles of 4 windows
  int slo[2], shi[2], ntile[2], own_lo[2], own_hi[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int bb = q == 0 ? b0 : b1i;
    const int ylo = max(0, R0 - 18 * bb - 2), yhi = min(13, R1 - 1 - 18 * bb - 2);
    const bool used = q == 0 || b1i != b0;
    slo[q] = ylo * 14;
    shi[q] = (used && yhi >= ylo) ? (yhi + 1) * 14 : slo[q];
    ntile[q] = (shi[q] - slo[q] + 3) / 4;
    const int wlo = max(gw0, 49 * bb) - 49 * bb, whi = min(gw1, 49 * bb + 48) - 49 * bb;  // conv2 windows
    own_lo[q] = 2 * (wlo / 7) * 14;
    own_hi[q] = (2 * (whi / 7) + 2) * 14;
  }
  const int nt_all = ntile[0] + ntile[1];
  for (int tl = wave; tl < nt_all; tl += 4) {  // wave-uniform
    const int q = tl < ntile[0] ? 0 : 1, tq = q == 0 ? tl : tl - ntile[0];
    const int bb = q == 0 ? b0 : b1i;
    const float* xs = xim + (bb - b0) * 1024;
    const int wa = min(slo[q] + 4 * tq + (lr >> 2), shi[q] - 1), d = lr & 3;
    const int pya = wa / 14, pxa = wa - pya * 14;
    const int base = (2 * pya + (d >> 1)) * 32 + 2 * pxa + (d & 1);
    float av[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) av[s] = xs[base + toff[s]];
    f32x4 cc0 = {0.f, 0.f, 0.f, 0.f}, cc1 = cc0;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      cc0 = mfma4(av[s], wb1[0][s], cc0);
      cc1 = mfma4(av[s], wb1[1][s], cc1);
    }
    const int win = slo[q] + 4 * tq + lg;
    if (win < shi[q]) {
      const int py = win / 14, px = win - py * 14;
      const int R = 18 * bb + py + 2 - R0;
      const bool own = win >= own_lo[q] && win < own_hi[q];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 c = nt ? cc1 : cc0;
        int best;
        const float m = pool4(c, best);
        const float v = fmaxf(m + (nt ? bias1 : bias0), 0.f);
        img[(R * C2F_RW + px + 2) * C2F_PS + 16 * nt + lr] = v;
        if (own) {
          const int64_t o = (((int64_t)bb * 14 + py) * 14 + px) * 32 + 16 * nt + lr;
          c1.a1[o] = v;
          c1.idx1[o] = (uint8_t)best;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ //
// conv2 forward, 8-wave form (MIHVD_F32_C2F_W8=1): the same tiles, image and epilogue, but 512
// threads: wave w = co group (w & 3) x ci half (w >> 2), so the two waves sharing a SIMD split K
// (25 taps x 16 channels each, 100 W2 floats per lane) and hide each other's LDS and MFMA latency
// instead of one wave per SIMD running the whole 800-deep chain; twice the threads stage the image.
// The two ci halves' accumulators meet in LDS behind the image (a fixed order: half 0 + half 1);
// the pool epilogue of the block's tiles is split between the halves.
// The image of this form: unpadded 32-float pixels in 18-pixel tall rows, each pixel's eight 16-byte
// chunks XOR-permuted by 2 ((row + column) & 3): the ds_read_b128 of every tap, tile and window-row
// wrap then lands its 16-lane groups on 16 distinct slots (scripts/ldssim_conv2.py model: 1.00 LDS
// cycles per group, against 1.42 for the padded 40 x 20 layout of the 4-wave form).
constexpr int C2F8_PS = 32, C2F8_RW = 18, C2F8_RS = C2F8_RW * C2F8_PS;
constexpr int C2F8_IMG = C2F_MAXR * C2F8_RS * 4;  // 50,688 B
__device__ __forceinline__ int c2f8_swz(int row, int col) { return ((row + col) & 3) << 1; }

// lane row lr of tile `tile`: pixel offset in the image (row * RW + col) * PS, and row + col
__device__ __forceinline__ int c2f8_base(int tile, int lr, int nwin, int R0, int& rc) {
  const int m = 16 * tile + lr;
  const int gw = min(m >> 2, nwin - 1), d = m & 3;
  const int bb = gw / 49, win = gw - 49 * bb, py = win / 7, px = win - 7 * py;
  const int r = 18 * bb + 2 * py + (d >> 1) - R0, x = 2 * px + (d & 1);
  rc = r + x;
  return (r * C2F8_RW + x) * C2F8_PS;
}

template <int NT, int DEPTH = 2>
__device__ __forceinline__ void c2f_tiles_h(const float* img, const int (&ab)[2], const int (&cw)[2][4],
                                            const float (&wb)[100], f32x4 (&acc)[2]) {
  constexpr int R = DEPTH + 1;
  float4 ra[R][NT];
  auto load_a = [&](float4 (&a)[NT], int tap) {
    const int kh = tap / 5, kw = tap - 5 * kh;
    const int off = (kh * C2F8_RW + kw) * C2F8_PS;
#pragma unroll
    for (int u = 0; u < NT; ++u) a[u] = *reinterpret_cast<const float4*>(img + ab[u] + off + cw[u][(kh + kw) & 3]);
  };
  auto mfma_step = [&](const float4 (&a)[NT], int tap) {
    const float* w = wb + 4 * tap;  // wb[4 tap + j]
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].x, w[0], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].y, w[1], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].z, w[2], acc[u]);
#pragma unroll
    for (int u = 0; u < NT; ++u) acc[u] = mfma4(a[u].w, w[3], acc[u]);
  };
#pragma unroll
  for (int st = 0; st < DEPTH; ++st) load_a(ra[st], st);
#pragma unroll
  for (int st = 0; st < 25; ++st) {
    if (st + DEPTH < 25) load_a(ra[(st + DEPTH) % R], st + DEPTH);
    __builtin_amdgcn_sched_barrier(0);
    mfma_step(ra[st % R], st);
    __builtin_amdgcn_sched_barrier(0);
  }
}

constexpr int C2F8_MAXCH = (C2F_MAXR * 18 * 8 + 511) / 512;  // image float4 chunks per thread
constexpr int C2F8_LDS = C2F8_IMG + 4 * 7 * 64 * 16;         // image + [co group][tile][lane] f32x4 exchange

template <int TPB, bool FRAG, int DEPTH = 2>
__global__ void __launch_bounds__(512) f32_conv2_fwd8_kernel(const float* __restrict__ a1, const float* __restrict__ w2,
                                                             const float* __restrict__ b2, float* __restrict__ a2,
                                                             uint8_t* __restrict__ idx2, int B,
                                                             const float* __restrict__ w2f, F32Adam ad) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  if ((int)blockIdx.x < ad.nblk) {  // optimizer tail blocks (MIHVD_F32_W3=tail), first in dispatch order
    f32_adam_stream(ad, blockIdx.x);
    return;
  }
  float* img = smf;
  f32x4* xr = reinterpret_cast<f32x4*>(smf + C2F8_IMG / 4);
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int wco = wave & 3, c2 = wave >> 2;
  // XCD-contiguous tile ranges: XCD x takes the images whose a1 rows conv1's blocks on XCD x wrote
  const int nblk = (((49 * B + 3) / 4) + TPB - 1) / TPB, lo = max(ad.nblk, 0);
  const int nwin = 49 * B, T0 = xcd_contiguous((int)blockIdx.x, lo, lo + nblk) * TPB;
  const int gw0 = 4 * T0, gw1 = min(4 * (T0 + TPB), nwin) - 1;
  const int b0 = gw0 / 49, b1i = gw1 / 49;
  const int R0 = 18 * b0 + 2 * ((gw0 - 49 * b0) / 7);
  const int R1 = 18 * b1i + 2 * ((gw1 - 49 * b1i) / 7) + 6;
  const int nch = (R1 - R0) * 144;  // 18 pixels x 8 float4 per tall row
  float4 iv[C2F8_MAXCH];
#pragma unroll
  for (int it = 0; it < C2F8_MAXCH; ++it) {
    const int i = min(t + 512 * it, nch - 1);
    const int rr = i / 144, rem = i - rr * 144, c = rem >> 3, ch = rem & 7;
    const int R = R0 + rr, bb = R / 18, y = R - 18 * bb - 2, xx = c - 2;
    const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
    const float4 v = *reinterpret_cast<const float4*>(
        a1 + (((int64_t)bb * 14 + (in ? y : 0)) * 14 + (in ? xx : 0)) * 32 + ch * 4);
    iv[it] = mask_f4(v, in);
  }
#pragma unroll
  for (int it = 0; it < C2F8_MAXCH; ++it) {
    const int i = t + 512 * it;
    if (i < nch) {
      const int rr = i / 144, rem = i - rr * 144, c = rem >> 3;
      *reinterpret_cast<float4*>(img + (rr * C2F8_RW + c) * C2F8_PS + 4 * ((rem & 7) ^ c2f8_swz(rr, c))) = iv[it];
    }
  }
  __syncthreads();  // the image is complete; no barrier below until the exchange
  // this wave's W2 operand: wb[4 tap + j] = W2[tap][16 c2 + 4 lg + j][16 wco + lr], consumed in issue order
  float wb[100];
  if constexpr (FRAG) {
    const float4* fp = reinterpret_cast<const float4*>(w2f) + (c2 * 4 + wco) * 64 + lane;
#pragma unroll
    for (int tap = 0; tap < 25; ++tap) {
      const float4 v = fp[tap * 512];
      wb[4 * tap + 0] = v.x;
      wb[4 * tap + 1] = v.y;
      wb[4 * tap + 2] = v.z;
      wb[4 * tap + 3] = v.w;
    }
  } else {
    const float* wp = w2 + (16 * c2 + 4 * lg) * 64 + 16 * wco + lr;
#pragma unroll
    for (int tap = 0; tap < 25; ++tap)
#pragma unroll
      for (int j = 0; j < 4; ++j) wb[4 * tap + j] = wp[tap * 2048 + j * 64];
  }
  f32x4 accs[TPB];
#pragma unroll
  for (int i = 0; i < TPB; i += 2) {  // block-uniform
    const int tile0 = T0 + i, tile1 = T0 + min(i + 1, TPB - 1);
    int rc0, rc1;
    const int ab[2] = {c2f8_base(tile0, lr, nwin, R0, rc0), c2f8_base(tile1, lr, nwin, R0, rc1)};
    // the lane's chunk 4 c2 + lg, swizzled for each (row + column) residue the taps visit
    int cw[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      cw[0][j] = 4 * ((4 * c2 + lg) ^ c2f8_swz(rc0 + j, 0));
      cw[1][j] = 4 * ((4 * c2 + lg) ^ c2f8_swz(rc1 + j, 0));
    }
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int nt = min(2, TPB - i);
    if (nt == 2) c2f_tiles_h<2, DEPTH>(img, ab, cw, wb, acc);
    else c2f_tiles_h<1, DEPTH>(img, ab, cw, wb, acc);
    accs[i] = acc[0];
    if (i + 1 < TPB) accs[i + 1] = acc[1];
  }
  // exchange: tile u is finished by ci half (u >= H): the other half hands over its partial
  constexpr int H = (TPB + 1) / 2;
#pragma unroll
  for (int u = 0; u < TPB; ++u)
    if ((u >= H) != (c2 == 1)) xr[(wco * 7 + u) * 64 + lane] = accs[u];
  __syncthreads();
  const int co = 16 * wco + lr;
  const float bias = b2[co];
#pragma unroll
  for (int u = 0; u < TPB; ++u) {
    if ((u >= H) != (c2 == 1)) continue;
    const f32x4 o = xr[(wco * 7 + u) * 64 + lane];
    const f32x4 sum = c2 == 0 ? accs[u] + o : o + accs[u];  // half 0 + half 1 either way
    const int gw = 4 * (T0 + u) + lg;
    if (gw < nwin) {
      const int bb = gw / 49, win = gw - 49 * bb;
      int best;
      const float m = pool4(sum, best);
      const int64_t oo = (int64_t)bb * 3136 + win * 64 + co;
      a2[oo] = fmaxf(m + bias, 0.f);
      idx2[oo] = (uint8_t)best;
    }
  }
}

// PREW: the W2 register operand is issued right behind the staging writes and the barrier orders
// LDS alone, so the 200 KB per block of W2 loads overlap the barrier wait and the first taps.
// FUSE1: the a1 rows are computed from x in the block (conv1 fused, C1Fuse) instead of loaded.
// FRAG: the W2 operand from the fragment copy (f32_w2_frag_block): 50 float4 loads per lane.
template <int TPB, bool TAIL, bool PREW = false, bool FUSE1 = false, int DEPTH = 2, bool FRAG = false>
__global__ void __launch_bounds__(256) f32_conv2_fwd_kernel(const float* __restrict__ a1, const float* __restrict__ w2,
                                                            const float* __restrict__ b2, float* __restrict__ a2,
                                                            uint8_t* __restrict__ idx2, int B, F32Adam ad, C1Fuse c1,
                                                            const float* __restrict__ w2f) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  if constexpr (TAIL) {
    if ((int)blockIdx.x < ad.nblk) {
      f32_adam_stream(ad, blockIdx.x);
      return;
    }
  }
  float* img = smf;
  c2f_stamp(0);
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int nwin = 49 * B, T0 = ((int)blockIdx.x - (TAIL ? ad.nblk : 0)) * TPB;
  const int gw0 = 4 * T0, gw1 = min(4 * (T0 + TPB), nwin) - 1;
  const int b0 = gw0 / 49, b1i = gw1 / 49;
  const int R0 = 18 * b0 + 2 * ((gw0 - 49 * b0) / 7);
  const int R1 = 18 * b1i + 2 * ((gw1 - 49 * b1i) / 7) + 6;
  const int nch = (R1 - R0) * 144;  // 18 pixels x 8 float4 per tall row
  if constexpr (FUSE1) {
    // 1. x of the (at most two) images into LDS, the tall image zeroed (its padding stays zero)
    float* xim = smf + C2F_MAXR * C2F_RS;
    int64_t step = c1.state ? c1.state[ST_FWD] : 0;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int i = t + 256 * it, sl = i >> 10, pix = i & 1023, Y = (pix >> 5) - 2, X = (pix & 31) - 2;
      const int bb = min(b0 + sl, B - 1);
      int row = bb;
      if (c1.rows != nullptr) row = c1.rows[(int)((step * (int64_t)B + bb) % c1.n_pool)];
      const bool in = Y >= 0 && Y < 28 && X >= 0 && X < 28;
      xim[i] = mask_f(c1.x[(int64_t)row * 784 + (in ? Y * 28 + X : 0)], in);
    }
    const int nz = (R1 - R0) * C2F_RS / 4;
    for (int i = t; i < nz; i += 256) reinterpret_cast<float4*>(img)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    __syncthreads();
    c2f_conv1_stage(c1, img, xim, B, R0, R1, b0, b1i, gw0, gw1);
  } else {
    // 1. the image rows
    float4 iv[C2F_MAXCH];
#pragma unroll
    for (int it = 0; it < C2F_MAXCH; ++it) {
      const int i = min(t + 256 * it, nch - 1);
      const int rr = i / 144, rem = i - rr * 144, c = rem >> 3, ch = rem & 7;
      const int R = R0 + rr, bb = R / 18, y = R - 18 * bb - 2, xx = c - 2;
      const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
      const float4 v = *reinterpret_cast<const float4*>(
          a1 + (((int64_t)bb * 14 + (in ? y : 0)) * 14 + (in ? xx : 0)) * 32 + ch * 4);
      iv[it] = mask_f4(v, in);
    }
#pragma unroll
    for (int it = 0; it < C2F_MAXCH; ++it) {
      const int i = t + 256 * it;
      if (i < nch) {
        const int rr = i / 144, rem = i - rr * 144;
        *reinterpret_cast<float4*>(img + (rr * C2F_RW + (rem >> 3)) * C2F_PS + (rem & 7) * 4) = iv[it];
      }
    }
  }
  float wb[200];  // wb[8 tap + 4 c2 + j] = W2[tap][16 c2 + 4 lg + j][16 w + lr]
  const float* wp = w2 + (4 * lg) * 64 + 16 * wave + lr;
  auto load_w = [&]() {
    if constexpr (FRAG) {
      const float4* fp = reinterpret_cast<const float4*>(w2f) + wave * 64 + lane;
#pragma unroll
      for (int s2 = 0; s2 < 50; ++s2) {
        const float4 v = fp[s2 * 256];
        wb[4 * s2 + 0] = v.x;
        wb[4 * s2 + 1] = v.y;
        wb[4 * s2 + 2] = v.z;
        wb[4 * s2 + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int tap = 0; tap < 25; ++tap)
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
          for (int j = 0; j < 4; ++j) wb[8 * tap + 4 * c2 + j] = wp[tap * 2048 + (16 * c2 + j) * 64];
    }
  };
  if constexpr (PREW) {
    __builtin_amdgcn_sched_barrier(0);
    load_w();
    __builtin_amdgcn_sched_barrier(0);
    c2f_lds_barrier();  // the image is complete; the W2 loads stay in flight
  } else {
    __syncthreads();  // the image is complete; no barrier below
    // the weights, issued after the barrier (whose vmcnt(0) would otherwise wait for all 200
    // loads): the MFMA steps consume them in issue order, each waiting only for its own
    load_w();
  }
  c2f_stamp(1);
  const int co = 16 * wave + lr;
  const float bias = b2[co];
  // unrolled: the first tile pair's MFMAs then wait for each W2 tap as it lands (a runtime loop
  // waits for every outstanding load at its entry)
#pragma unroll
  for (int i = 0; i < TPB; i += 2) {  // block-uniform
    const int tile0 = T0 + i, tile1 = T0 + min(i + 1, TPB - 1);
    const int ab[2] = {c2f_abase(tile0, lr, lg, nwin, R0), c2f_abase(tile1, lr, lg, nwin, R0)};
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    const int nt = min(2, TPB - i);
    if (nt == 2) c2f_tiles<2, DEPTH>(img, ab, wb, acc);
    else c2f_tiles<1, DEPTH>(img, ab, wb, acc);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int gw = 4 * (T0 + i + u) + lg;
      if (u < nt && gw < nwin) {
        const int bb = gw / 49, win = gw - 49 * bb;
        int best;
        const float m = pool4(acc[u], best);
        const int64_t o = (int64_t)bb * 3136 + win * 64 + co;
        a2[o] = fmaxf(m + bias, 0.f);
        idx2[o] = (uint8_t)best;
      }
    }
    c2f_stamp(2 + (i >> 1));
  }
}

// ------------------------------------------------------------------------------------------ //
// fc1 forward: zpart[ks][b][n] = sum_{k in slice ks} a2[b][k] W3[k][n]   (14 slices of 224)
// grid (16, 14): 64 columns x one K slice per block, 8 waves: wave w = 16 columns (w & 3) x every
// other 16-sample tile (w >> 2). The transposed product puts features on the MFMA row axis: A =
// W3^T, whose 56 fragments for the slice (one W3 element per lane per MFMA) are loaded once into
// registers straight from HBM (every W3 element is read by one block); B = a2^T from the slice's
// K-contiguous LDS image (one float4 per 4 MFMAs). A lane's 4 accumulators are 4 consecutive
// features of one sample: 16-byte slab stores.
// ------------------------------------------------------------------------------------------ //
// a2 slice row stride 232 floats (58 16-byte slots, = 2 mod 4): the B-operand ds_read_b128 of lane
// (lr, lg) at slot 58 lr + lg covers 16 distinct slots in each 16-lane group (scripts/ldssim_conv2.py
// model: 1.0 LDS cycles per group; 228 gave 2.0, PMC LDS_BANK_CONFLICT 1.7x the active LDS cycles)
constexpr int F1F_KS = 14, F1F_KSL = 224, F1F_AS = 232;
constexpr int F1F_LDS = 128 * F1F_AS * 4;  // 118,784 B

// ADAM: dense/kernel's deferred Adam update (the previous step's gradient) is applied here, where
// W3 is read anyway (one read of p instead of two): the block first streams Adam over its
// [224 k][64 n] tile of W3 with coalesced float4 accesses (p, g, m, v in; p, m, v out), keeps the
// new tile in LDS and takes the MFMA fragments from there. Every W3 element belongs to exactly one
// block. LDS: the a2 slice + the tile, so MT <= 7 (B <= 112).
constexpr int F1F_WS = 64;                          // W3 tile row stride in LDS (floats)
constexpr int F1F_LDS_ADAM = 7 * 16 * F1F_AS * 4 + F1F_KSL * F1F_WS * 4;   // 161,280 B
static_assert(F1F_LDS_ADAM <= 163840, "fc1 forward with the fused update: LDS");

template <int MT, bool ADAM>
__global__ void __launch_bounds__(512) f32_fc1_fwd_kernel(const float* __restrict__ a2, float* __restrict__ w3,
                                                          float* __restrict__ zpart, int B, F32Adam ad) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* As = smf;  // [16 MT][228]: rows = samples, k contiguous
  const int nb = blockIdx.x, ks = blockIdx.y, t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int k0 = ks * F1F_KSL, nt = wave & 3, sh = wave >> 2;
  const int n = nb * 64 + nt * 16 + lr;
  constexpr int NCH = MT * 16 * 56, PER = (NCH + 511) / 512;
  float wa[56];  // A fragments: wa[4q + j] = W3[k0 + 16q + 4lg + j][n]
  const int64_t wo = (int64_t)(k0 + 4 * lg) * 1024 + n;
  if constexpr (ADAM) {
    static_assert(MT <= 7, "the fused update needs the a2 slice and the W3 tile in LDS");
    float* Ws = smf + 7 * 16 * F1F_AS;  // [224][64]: the updated tile
    const AdamCoef c = f32_adam_coef(ad);
    // tile float4 i (0..3583): row i >> 4, float4 column i & 15; 7 per thread, all 28 loads in flight
    float4 pv[7], gv[7], mv[7], vv[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int i = t + 512 * u;
      const int64_t o = (int64_t)(k0 + (i >> 4)) * 1024 + nb * 64 + 4 * (i & 15);
      pv[u] = *reinterpret_cast<const float4*>(w3 + o);
      gv[u] = *reinterpret_cast<const float4*>(ad.g + o);
      mv[u] = *reinterpret_cast<const float4*>(ad.m + o);
      vv[u] = *reinterpret_cast<const float4*>(ad.v + o);
    }
    float4 v[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = min(t + 512 * it, NCH - 1), r = i / 56, cc = i - 56 * r;
      v[it] = mask_f4(*reinterpret_cast<const float4*>(a2 + (int64_t)min(r, B - 1) * 3136 + k0 + 4 * cc), r < B);
    }
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int i = t + 512 * u;
      const int64_t o = (int64_t)(k0 + (i >> 4)) * 1024 + nb * 64 + 4 * (i & 15);
      adam4_f32(pv[u], mv[u], vv[u], gv[u], c);
      *reinterpret_cast<float4*>(w3 + o) = pv[u];
      *reinterpret_cast<float4*>(ad.m + o) = mv[u];
      *reinterpret_cast<float4*>(ad.v + o) = vv[u];
      *reinterpret_cast<float4*>(Ws + (i >> 4) * F1F_WS + 4 * (i & 15)) = pv[u];
    }
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = t + 512 * it;
      if (i < NCH) {
        const int r = i / 56, cc = i - 56 * r;
        *reinterpret_cast<float4*>(As + r * F1F_AS + 4 * cc) = v[it];
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 14; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[4 * q + j] = Ws[(16 * q + 4 * lg + j) * F1F_WS + nt * 16 + lr];
  } else {
#pragma unroll
    for (int q = 0; q < 14; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[4 * q + j] = w3[wo + (16 * q + j) * 1024];
    float4 v[PER];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = min(t + 512 * it, NCH - 1), r = i / 56, cc = i - 56 * r;
      v[it] = mask_f4(*reinterpret_cast<const float4*>(a2 + (int64_t)min(r, B - 1) * 3136 + k0 + 4 * cc), r < B);
    }
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = t + 512 * it;
      if (i < NCH) {
        const int r = i / 56, cc = i - 56 * r;
        *reinterpret_cast<float4*>(As + r * F1F_AS + 4 * cc) = v[it];
      }
    }
    __syncthreads();
  }
  for (int tt = sh; tt < MT; tt += 2) {  // wave-uniform
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    const float* bp = As + (tt * 16 + lr) * F1F_AS + 4 * lg;
#pragma unroll
    for (int q = 0; q < 14; q += 2) {
      const float4 b0 = *reinterpret_cast<const float4*>(bp + 16 * q);
      const float4 b1 = *reinterpret_cast<const float4*>(bp + 16 * q + 16);
      acc0 = mfma4_q(make_float4(wa[4 * q], wa[4 * q + 1], wa[4 * q + 2], wa[4 * q + 3]), b0, acc0);
      acc1 = mfma4_q(make_float4(wa[4 * q + 4], wa[4 * q + 5], wa[4 * q + 6], wa[4 * q + 7]), b1, acc1);
    }
    const int m = tt * 16 + lr;
    if (m < B) {
      const f32x4 s = acc0 + acc1;
      *reinterpret_cast<float4*>(zpart + ((int64_t)ks * B + m) * 1024 + nb * 64 + nt * 16 + 4 * lg) =
          make_float4(s[0], s[1], s[2], s[3]);
    }
  }
}

// fc1 forward, pipelined form (default; MIHVD_F32_F1F=0 selects the form above). Same grid,
// slabs and operand layouts; two changes:
//  * MFMA core: a wave's NT tiles (sh, sh + 2, ...) are interleaved element-outer, tile-inner, so
//    dependent MFMAs sit NT issues apart (the form above alternated two accumulators: 2 x 32 cycles
//    against the 40-cycle dependent latency), and the a2 chunks are read from LDS two chunks ahead.
//  * ADAM: the update streams in 7 parts of 32 rows (one float4 of p/g/m/v per thread per part);
//    part p + 1's update and part p + 2's loads run while the MFMAs of part p issue, so the HBM
//    stream and the matrix cores overlap instead of taking turns (the form above applied the whole
//    tile's update, then ran every MFMA).
template <int NT, int Q0, int Q1>
__device__ __forceinline__ void f1f_mma(const float (&wa)[56], const float* __restrict__ bp, f32x4 (&acc)[4]) {
  if constexpr (NT > 0) {
    constexpr int NQ = Q1 - Q0, DQ = 2, R = DQ + 1;
    float4 bq[R][NT];
#pragma unroll
    for (int j = 0; j < DQ; ++j)
      if (j < NQ) {
#pragma unroll
        for (int u = 0; u < NT; ++u) bq[j][u] = *reinterpret_cast<const float4*>(bp + u * 32 * F1F_AS + 16 * (Q0 + j));
      }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      if (j + DQ < NQ) {
#pragma unroll
        for (int u = 0; u < NT; ++u)
          bq[(j + DQ) % R][u] = *reinterpret_cast<const float4*>(bp + u * 32 * F1F_AS + 16 * (Q0 + j + DQ));
      }
      __builtin_amdgcn_sched_barrier(0);
      const int q = Q0 + j, s = j % R;
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[u] = mfma4(wa[4 * q + 0], bq[s][u].x, acc[u]);
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[u] = mfma4(wa[4 * q + 1], bq[s][u].y, acc[u]);
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[u] = mfma4(wa[4 * q + 2], bq[s][u].z, acc[u]);
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[u] = mfma4(wa[4 * q + 3], bq[s][u].w, acc[u]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// SPLIT (no ADAM): the a2 slice is staged in two K halves of 112: the second half's loads (and its
// W3 fragments) are in flight while the MFMAs of the first half issue, instead of every MFMA waiting
// for the whole 100 KB slice.
template <int MT, bool ADAM, bool SPLIT = false>
__global__ void __launch_bounds__(512) f32_fc1_fwd2_kernel(const float* __restrict__ a2, float* __restrict__ w3,
                                                           float* __restrict__ zpart, int B, F32Adam ad) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* As = smf;  // [16 MT][228]: rows = samples, k contiguous
  const int nb = blockIdx.x, ks = blockIdx.y, t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int k0 = ks * F1F_KSL, nt = wave & 3, sh = wave >> 2;
  const int n = nb * 64 + nt * 16 + lr;
  constexpr int NCH = MT * 16 * 56, PER = (NCH + 511) / 512;
  constexpr int NT0 = (MT + 1) / 2, NT1 = MT / 2;  // tiles of the sh = 0 / sh = 1 waves
  const float* bp = As + (sh * 16 + lr) * F1F_AS + 4 * lg;
  float wa[56];  // A fragments: wa[4q + j] = W3[k0 + 16q + 4lg + j][n]
  f32x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (SPLIT) {
    static_assert(!ADAM, "the split staging is the plain forward's");
    constexpr int NCH2 = MT * 16 * 28, PER2 = (NCH2 + 511) / 512;  // one K half: 28 float4 per row
    float4 v0[PER2], v1[PER2];
    auto ld_half = [&](float4 (&v)[PER2], int h) {
#pragma unroll
      for (int it = 0; it < PER2; ++it) {
        const int i = min(t + 512 * it, NCH2 - 1), r = i / 28, cc = 28 * h + i - 28 * r;
        v[it] = mask_f4(*reinterpret_cast<const float4*>(a2 + (int64_t)min(r, B - 1) * 3136 + k0 + 4 * cc), r < B);
      }
    };
    auto st_half = [&](const float4 (&v)[PER2], int h) {
#pragma unroll
      for (int it = 0; it < PER2; ++it) {
        const int i = t + 512 * it;
        if (i < NCH2) {
          const int r = i / 28, cc = 28 * h + i - 28 * r;
          *reinterpret_cast<float4*>(As + r * F1F_AS + 4 * cc) = v[it];
        }
      }
    };
    const int64_t wo = (int64_t)(k0 + 4 * lg) * 1024 + n;
    auto ld_w = [&](int q0, int q1) {
#pragma unroll
      for (int q = q0; q < q1; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) wa[4 * q + j] = w3[wo + (16 * q + j) * 1024];
    };
    // issue order (pinned): a2 half 0, W3 q 0..6, a2 half 1, W3 q 7..13 — the in-order load counter
    // then lets half 0's writes and MFMAs wait for their own operands only
    ld_half(v0, 0);
    __builtin_amdgcn_sched_barrier(0);
    ld_w(0, 7);
    __builtin_amdgcn_sched_barrier(0);
    ld_half(v1, 1);
    __builtin_amdgcn_sched_barrier(0);
    ld_w(7, 14);
    __builtin_amdgcn_sched_barrier(0);
    st_half(v0, 0);
    c2f_lds_barrier();
    if (sh == 0)
      f1f_mma<NT0, 0, 7>(wa, bp, acc);
    else
      f1f_mma<NT1, 0, 7>(wa, bp, acc);
    st_half(v1, 1);  // K columns the first half's reads never touch
    c2f_lds_barrier();
    if (sh == 0)
      f1f_mma<NT0, 7, 14>(wa, bp, acc);
    else
      f1f_mma<NT1, 7, 14>(wa, bp, acc);
    const int ntl = sh == 0 ? NT0 : NT1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int tt = sh + 2 * u, m = tt * 16 + lr;
      if (u < ntl && m < B)
        *reinterpret_cast<float4*>(zpart + ((int64_t)ks * B + m) * 1024 + nb * 64 + nt * 16 + 4 * lg) =
            make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
    }
    return;
  }
  float4 v[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = min(t + 512 * it, NCH - 1), r = i / 56, cc = i - 56 * r;
    v[it] = mask_f4(*reinterpret_cast<const float4*>(a2 + (int64_t)min(r, B - 1) * 3136 + k0 + 4 * cc), r < B);
  }
  if constexpr (!ADAM) {
    const int64_t wo = (int64_t)(k0 + 4 * lg) * 1024 + n;
#pragma unroll
    for (int q = 0; q < 14; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[4 * q + j] = w3[wo + (16 * q + j) * 1024];
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = t + 512 * it;
      if (i < NCH) {
        const int r = i / 56, cc = i - 56 * r;
        *reinterpret_cast<float4*>(As + r * F1F_AS + 4 * cc) = v[it];
      }
    }
    // LDS-only barrier: the W3 fragments (issued before the a2 writes, read from HBM) stay in
    // flight; the MFMA chain consumes them in issue order
    c2f_lds_barrier();
    if (sh == 0)
      f1f_mma<NT0, 0, 14>(wa, bp, acc);
    else
      f1f_mma<NT1, 0, 14>(wa, bp, acc);
  } else {
    static_assert(MT <= 7, "the fused update needs the a2 slice and the W3 tile in LDS");
    float* Ws = smf + 7 * 16 * F1F_AS;  // [224][64]: the updated tile
    const AdamCoef c = f32_adam_coef(ad);
    // part p: rows [32 p, 32 p + 32) of the slice; thread t owns row 32 p + (t >> 4), float4 column t & 15
    const int64_t o0 = (int64_t)(k0 + (t >> 4)) * 1024 + nb * 64 + 4 * (t & 15);
    float* wsp = Ws + (t >> 4) * F1F_WS + 4 * (t & 15);
    float4 P[3], Gv[3], M[3], V[3];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int64_t o = o0 + (int64_t)p * 32 * 1024;
      P[p] = *reinterpret_cast<const float4*>(w3 + o);
      Gv[p] = *reinterpret_cast<const float4*>(ad.g + o);
      M[p] = *reinterpret_cast<const float4*>(ad.m + o);
      V[p] = *reinterpret_cast<const float4*>(ad.v + o);
    }
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = t + 512 * it;
      if (i < NCH) {
        const int r = i / 56, cc = i - 56 * r;
        *reinterpret_cast<float4*>(As + r * F1F_AS + 4 * cc) = v[it];
      }
    }
    auto update = [&](int p, int s) {
      const int64_t o = o0 + (int64_t)p * 32 * 1024;
      adam4_f32(P[s], M[s], V[s], Gv[s], c);
      *reinterpret_cast<float4*>(w3 + o) = P[s];
      *reinterpret_cast<float4*>(ad.m + o) = M[s];
      *reinterpret_cast<float4*>(ad.v + o) = V[s];
      *reinterpret_cast<float4*>(wsp + p * 32 * F1F_WS) = P[s];
    };
    update(0, 0);
    __syncthreads();
    // part p (compile-time, so the q range of the MFMA core is static)
    auto part = [&](auto pc) {
      constexpr int p = decltype(pc)::value;
      if constexpr (p + 2 < 7) {
        constexpr int s = (p + 2) % 3;
        const int64_t o = o0 + (int64_t)(p + 2) * 32 * 1024;
        P[s] = *reinterpret_cast<const float4*>(w3 + o);
        Gv[s] = *reinterpret_cast<const float4*>(ad.g + o);
        M[s] = *reinterpret_cast<const float4*>(ad.m + o);
        V[s] = *reinterpret_cast<const float4*>(ad.v + o);
      }
#pragma unroll
      for (int q = 2 * p; q < 2 * p + 2; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) wa[4 * q + j] = Ws[(16 * q + 4 * lg + j) * F1F_WS + nt * 16 + lr];
      if (sh == 0)
        f1f_mma<NT0, 2 * p, 2 * p + 2>(wa, bp, acc);
      else
        f1f_mma<NT1, 2 * p, 2 * p + 2>(wa, bp, acc);
      if constexpr (p + 1 < 7) update(p + 1, (p + 1) % 3);
      __syncthreads();
    };
    part(std::integral_constant<int, 0>{});
    part(std::integral_constant<int, 1>{});
    part(std::integral_constant<int, 2>{});
    part(std::integral_constant<int, 3>{});
    part(std::integral_constant<int, 4>{});
    part(std::integral_constant<int, 5>{});
    part(std::integral_constant<int, 6>{});
  }
  const int ntl = sh == 0 ? NT0 : NT1;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int tt = sh + 2 * u, m = tt * 16 + lr;
    if (u < ntl && m < B)
      *reinterpret_cast<float4*>(zpart + ((int64_t)ks * B + m) * 1024 + nb * 64 + nt * 16 + 4 * lg) =
          make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
  }
}

// ------------------------------------------------------------------------------------------ //
// head: one block per sample b, 256 threads x 4 features (K9-K11 of SURVEY.md §2.5):
//   z = sum of the 14 slabs + b3; h = dropout(relu(z)); logits = h W4 + b4; softmax-xent;
//   dlogits = (softmax - onehot) / B; dz = (dlogits W4^T) * relu'(z) * dropout mask
// ------------------------------------------------------------------------------------------ //
__global__ void __launch_bounds__(256) f32_head_kernel(
    const float* __restrict__ zpart, const float* __restrict__ b3, const float* __restrict__ w4,
    const float* __restrict__ b4, const int64_t* __restrict__ labels, const int* __restrict__ rows, int n_pool,
    int64_t* __restrict__ state, uint32_t seed, uint32_t thresh24, float keep_scale, float* __restrict__ h_out,
    float* __restrict__ dz_out, float* __restrict__ dlog_out, float* __restrict__ stats, int B) {
  __shared__ float red[4][10];
  __shared__ float dl[10];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t step = state ? state[ST_FWD] : 0;
  const int n0 = t * 4;
  float4 parts[F1F_KS];
#pragma unroll
  for (int s = 0; s < F1F_KS; ++s)
    parts[s] = *reinterpret_cast<const float4*>(zpart + ((int64_t)s * B + b) * 1024 + n0);
  float w4r[4][10];  // this thread's 4 rows of W4 = 40 contiguous floats
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
  int y = 0;
  if (t < 64) {
    int row = b;
    if (rows != nullptr) row = rows[(int)((step * (int64_t)B + b) % n_pool)];
    y = (int)labels[row];
  }
  float z[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
  for (int s = 0; s < F1F_KS; ++s) {
    z[0] += parts[s].x;
    z[1] += parts[s].y;
    z[2] += parts[s].z;
    z[3] += parts[s].w;
  }
  float h[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool keep = thresh24 == 0 || dropout_keep(seed, (uint32_t)step, (uint32_t)(b * 1024 + n0 + i), thresh24);
    h[i] = keep ? fmaxf(z[i], 0.f) * keep_scale : 0.f;
  }
  *reinterpret_cast<float4*>(h_out + (int64_t)b * 1024 + n0) = make_float4(h[0], h[1], h[2], h[3]);
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
    const int c = min(lane, 9);
    const float lgt = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]) + b4[c];
    const float v = lane < 10 ? lgt : -INFINITY;
    const float mx = wave_max(v);
    const float e = lane < 10 ? expf(lgt - mx) : 0.f;
    const float se = wave_sum(e);
    const float lse = mx + logf(se);
    const unsigned long long ismax = __ballot(lane < 10 && lgt == mx);
    const int am = __ffsll((long long)ismax) - 1;
    const float ly = __shfl(lgt, y, 64);
    if (lane < 10) {
      const float d = (expf(lgt - lse) - (lane == y ? 1.f : 0.f)) / (float)B;
      dl[lane] = d;
      dlog_out[b * 10 + lane] = d;
    }
    if (lane == 0) {
      stats[b * 2 + 0] = lse - ly;
      stats[b * 2 + 1] = (am == y) ? 1.f : 0.f;
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
    g[i] = h[i] > 0.f ? s * keep_scale : 0.f;
  }
  *reinterpret_cast<float4*>(dz_out + (int64_t)b * 1024 + n0) = make_float4(g[0], g[1], g[2], g[3]);
}

// ------------------------------------------------------------------------------------------ //
// host wrappers
// ------------------------------------------------------------------------------------------ //
static void check_f32(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kFloat && t.is_contiguous() && t.numel() == numel, what,
              ": expected a contiguous fp32 device tensor of ", numel, " elements");
}
static void check_u8(const at::Tensor& t, int64_t numel, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.dtype() == at::kByte && t.is_contiguous() && t.numel() == numel, what,
              ": expected a contiguous uint8 device tensor of ", numel, " elements");
}

static const int* rows_ptr(const c10::optional<at::Tensor>& rows, int n_pool, int B, const char* what) {
  if (rows.has_value() && rows->defined()) {
    TORCH_CHECK(rows->dtype() == at::kInt && rows->numel() == n_pool, what, ": rows must be int32 [n_pool]");
    return rows->data_ptr<int>();
  }
  TORCH_CHECK(n_pool >= B, what, ": x has fewer rows than the batch");
  return nullptr;
}

void f32_conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                   const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1,
                   const c10::optional<at::Tensor>& w2, const c10::optional<at::Tensor>& w2frag) {
  const int B = a1.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_conv1_fwd: batch 1..128");
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "f32_conv1_fwd: x");
  check_f32(a1, (int64_t)B * 6272, "f32_conv1_fwd: a1");
  check_u8(idx1, (int64_t)B * 6272, "f32_conv1_fwd: idx1");
  check_f32(w1, 800, "f32_conv1_fwd: w1");
  check_f32(b1, 32, "f32_conv1_fwd: b1");
  const int n_pool = x.size(0);
  const int* rp = rows_ptr(rows, n_pool, B, "f32_conv1_fwd");
  const int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  // with w2 and w2frag: 4 x 7 more blocks write the W2 fragment copies for the conv2 launches
  const bool frag = w2.has_value() && w2->defined() && w2frag.has_value() && w2frag->defined();
  if (frag) {
    check_f32(*w2, 51200, "f32_conv1_fwd: w2");
    check_f32(*w2frag, 2 * 51200, "f32_conv1_fwd: w2frag [2][51200]");
  }
  f32_conv1_kernel<<<dim3(4 * B + (frag ? 4 * W2F_BLOCKS_Y : 0)), 256, 0, stream>>>(
      x.data_ptr<float>(), rp, n_pool, sp, w1.data_ptr<float>(), b1.data_ptr<float>(), a1.data_ptr<float>(),
      idx1.data_ptr<uint8_t>(), B, frag ? w2->data_ptr<float>() : nullptr, frag ? w2frag->data_ptr<float>() : nullptr);
}

// tiles per block of f32_conv2_fwd for batch B (about one block per CU), and the block count
static int conv2f_tpb(int B) {
  const int nt = (49 * B + 3) / 4;
  return std::min(7, std::max(1, (nt + 255) / 256));
}

// Adam operands of a flat fp32 range (p, g, m, v: same length, multiple of 4) for a fused update;
// nblk = 0 when p is absent.
static F32Adam f32_adam_args(const c10::optional<at::Tensor>& p, const c10::optional<at::Tensor>& g,
                             const c10::optional<at::Tensor>& m, const c10::optional<at::Tensor>& v,
                             const c10::optional<at::Tensor>& state, double lr, double b1, double b2, double eps,
                             double gscale, int64_t rule, int nblk, const char* what) {
  F32Adam a;
  if (!(p.has_value() && p->defined())) return a;
  TORCH_CHECK(g.has_value() && m.has_value() && v.has_value() && state.has_value() && state->defined(), what,
              ": fused Adam needs p, g, m, v and the step state");
  const int64_t n = p->numel();
  for (const at::Tensor* t : {&*p, &*g, &*m, &*v})
    TORCH_CHECK(t->is_cuda() && t->dtype() == at::kFloat && t->is_contiguous() && t->numel() == n &&
                    ((uintptr_t)t->data_ptr() & 15) == 0,
                what, ": Adam operands must be 16-byte aligned contiguous fp32 tensors of one length");
  TORCH_CHECK(n % 4 == 0, what, ": Adam range must be a multiple of 4 elements");
  a.p = p->data_ptr<float>();
  a.g = g->data_ptr<float>();
  a.m = m->data_ptr<float>();
  a.v = v->data_ptr<float>();
  a.n4 = n / 4;
  a.state = state->data_ptr<int64_t>();
  a.lr = (float)lr;
  a.b1 = (float)b1;
  a.b2 = (float)b2;
  a.eps = (float)eps;
  a.gscale = (float)gscale;
  a.rule = (int)rule;
  a.nblk = nblk;
  return a;
}

static void f32_conv2_fwd_impl(const at::Tensor& a1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& a2,
                               at::Tensor& idx2, const c10::optional<at::Tensor>& p3,
                               const c10::optional<at::Tensor>& g3, const c10::optional<at::Tensor>& m3,
                               const c10::optional<at::Tensor>& v3, const c10::optional<at::Tensor>& state, double lr,
                               double beta1, double beta2, double eps, double grad_scale, int64_t rule,
                               int64_t tail_blocks, const C1Fuse& c1, const float* w2f);

void f32_conv2_fwd(const at::Tensor& a1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2,
                   const c10::optional<at::Tensor>& p3, const c10::optional<at::Tensor>& g3,
                   const c10::optional<at::Tensor>& m3, const c10::optional<at::Tensor>& v3,
                   const c10::optional<at::Tensor>& state, double lr, double beta1, double beta2, double eps,
                   double grad_scale, int64_t rule, int64_t tail_blocks, const c10::optional<at::Tensor>& w2frag) {
  const float* w2f = nullptr;
  if (w2frag.has_value() && w2frag->defined()) {
    TORCH_CHECK(w2frag->is_cuda() && w2frag->dtype() == at::kFloat && w2frag->is_contiguous() &&
                    w2frag->numel() >= 51200, "f32_conv2_fwd: w2frag (the forward fragment copy, 51200 floats)");
    w2f = w2frag->data_ptr<float>();
  }
  f32_conv2_fwd_impl(a1, w2, b2, a2, idx2, p3, g3, m3, v3, state, lr, beta1, beta2, eps, grad_scale, rule, tail_blocks,
                     C1Fuse{}, w2f);
}

// conv1 + conv2 forward in one launch: every conv2 block computes the a1 rows it reads from x (see
// c2f_conv1_stage); a1 / idx1 are written for the backward.
void f32_conv12_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                    const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1, const at::Tensor& w2,
                    const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2) {
  const int B = a1.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_conv12_fwd: batch 1..128");
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "f32_conv12_fwd: x");
  check_f32(a1, (int64_t)B * 6272, "f32_conv12_fwd: a1");
  check_u8(idx1, (int64_t)B * 6272, "f32_conv12_fwd: idx1");
  check_f32(w1, 800, "f32_conv12_fwd: w1");
  check_f32(b1, 32, "f32_conv12_fwd: b1");
  C1Fuse c1;
  c1.n_pool = x.size(0);
  c1.rows = rows_ptr(rows, c1.n_pool, B, "f32_conv12_fwd");
  c1.x = x.data_ptr<float>();
  c1.state = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  c1.w1 = w1.data_ptr<float>();
  c1.b1 = b1.data_ptr<float>();
  c1.a1 = a1.data_ptr<float>();
  c1.idx1 = idx1.data_ptr<uint8_t>();
  f32_conv2_fwd_impl(a1, w2, b2, a2, idx2, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, c10::nullopt, 0.0,
                     0.0, 0.0, 0.0, 1.0, 0, 0, c1, nullptr);
}

static void f32_conv2_fwd_impl(const at::Tensor& a1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& a2,
                               at::Tensor& idx2, const c10::optional<at::Tensor>& p3,
                               const c10::optional<at::Tensor>& g3, const c10::optional<at::Tensor>& m3,
                               const c10::optional<at::Tensor>& v3, const c10::optional<at::Tensor>& state, double lr,
                               double beta1, double beta2, double eps, double grad_scale, int64_t rule,
                               int64_t tail_blocks, const C1Fuse& c1, const float* w2f) {
  const bool fuse1 = c1.x != nullptr;
  const int B = a2.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_conv2_fwd: batch 1..128");
  check_f32(a1, (int64_t)B * 6272, "f32_conv2_fwd: a1");
  check_f32(w2, 51200, "f32_conv2_fwd: w2");
  check_f32(b2, 64, "f32_conv2_fwd: b2");
  check_f32(a2, (int64_t)B * 3136, "f32_conv2_fwd: a2");
  check_u8(idx2, (int64_t)B * 3136, "f32_conv2_fwd: idx2");
  const int tpb = conv2f_tpb(B), nt = (49 * B + 3) / 4, nblk = (nt + tpb - 1) / tpb;
  // every block's tall-row span must fit the LDS image (host check of the kernel's assumption)
  for (int blk = 0; blk < nblk; ++blk) {
    const int gw0 = 4 * blk * tpb, gw1 = std::min(4 * (blk + 1) * tpb, 49 * B) - 1;
    const int r0 = 18 * (gw0 / 49) + 2 * ((gw0 % 49) / 7), r1 = 18 * (gw1 / 49) + 2 * ((gw1 % 49) / 7) + 6;
    TORCH_CHECK(r1 - r0 <= C2F_MAXR, "f32_conv2_fwd: row span exceeds the LDS image");
  }
  const int nt_tail = tail_blocks > 0 ? (int)tail_blocks : device_cu_count();
  const F32Adam ad =
      f32_adam_args(p3, g3, m3, v3, state, lr, beta1, beta2, eps, grad_scale, rule, nt_tail, "f32_conv2_fwd");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  // When the grid fits the CUs, request more LDS than the image needs (> half a CU's) so no two
  // blocks share a CU: the dispatcher otherwise doubles blocks up on some CUs while others idle
  // (measured 20.6 -> 19.7 us at B = 100). MIHVD_F32_C2F_LDS overrides (study knob).
  const int spread = (nblk + (ad.nblk > 0 ? ad.nblk : 0)) <= device_cu_count() ? 81920 + 1024 : 0;
  const int need = C2F_LDS + (fuse1 ? C2F_XIM * 4 : 0);
  const int lds = std::max(need, std::min(env_knob("MIHVD_F32_C2F_LDS", spread), 163840));
  auto launch = [&](auto kern, int extra) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kern<<<nblk + extra, 256, lds, stream>>>(a1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(),
                                                 a2.data_ptr<float>(), idx2.data_ptr<uint8_t>(), B, ad, c1, w2f);
  };
  // MIHVD_F32_C2F_PREW=1: the W2 operand issued before the staging barrier (LDS-only barrier)
  // instead of after it. Measured slower standalone (21.0 vs 19.6 us: the 200 KB of W2 per block
  // then competes with the a1 staging loads at kernel start) and neutral in the whole step
  // (profiles/r04/kbench_f32_r04j.txt), so W2 follows a full barrier by default.
  const bool prew = env_knob("MIHVD_F32_C2F_PREW", 0) != 0;
  // MIHVD_F32_C2F_DEPTH=1: A reads one step ahead of the MFMAs instead of two (the earlier form)
  const bool shallow = env_knob("MIHVD_F32_C2F_DEPTH", 2) < 2;
  // MIHVD_F32_C2F_W8=1 (default): the 8-wave form (two ci halves per co group, f32_conv2_fwd8_kernel):
  // 18.9 vs 19.2 us with the fragment W2, whole step 122.6 vs 122.9 us (profiles/r04/kbench_f32_r04s.txt)
  const bool w8 = !fuse1 && !prew && env_knob("MIHVD_F32_C2F_W8", 1) != 0;
  if (w8) {
    TORCH_CHECK(tpb <= 7, "f32_conv2_fwd: 8-wave form needs <= 7 tiles per block");
    // (more LDS than a CU's half when the grid fits the CUs: one block per CU, as the 4-wave form)
    const int lds8 = std::max(C2F8_LDS, std::min(env_knob("MIHVD_F32_C2F_LDS", spread), 163840));
    auto launch8 = [&](auto kern) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds8);
      kern<<<nblk + std::max(ad.nblk, 0), 512, lds8, stream>>>(
          a1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(), a2.data_ptr<float>(),
          idx2.data_ptr<uint8_t>(), B, w2f, ad);
    };
#define C2F8_CASE(T)                                                                           \
  case T:                                                                                      \
    if (shallow) w2f ? launch8(f32_conv2_fwd8_kernel<T, true, 1>) : launch8(f32_conv2_fwd8_kernel<T, false, 1>); \
    else w2f ? launch8(f32_conv2_fwd8_kernel<T, true>) : launch8(f32_conv2_fwd8_kernel<T, false>);         \
    break;
    switch (tpb) {
      C2F8_CASE(1)
      C2F8_CASE(2)
      C2F8_CASE(3)
      C2F8_CASE(4)
      C2F8_CASE(5)
      C2F8_CASE(6)
      default:
        C2F8_CASE(7)
    }
#undef C2F8_CASE
    return;
  }
  TORCH_CHECK(!(fuse1 && ad.nblk > 0), "f32_conv2_fwd: the fused conv1 has no optimizer tail");
#define C2F_CASE(T)                                                                  \
  case T:                                                                            \
    if (ad.nblk > 0) launch(f32_conv2_fwd_kernel<T, true>, ad.nblk);                 \
    else if (fuse1) launch(f32_conv2_fwd_kernel<T, false, true, true>, 0);           \
    else if (prew) launch(f32_conv2_fwd_kernel<T, false, true>, 0);                  \
    else if (shallow && w2f) launch(f32_conv2_fwd_kernel<T, false, false, false, 1, true>, 0); \
    else if (shallow) launch(f32_conv2_fwd_kernel<T, false, false, false, 1>, 0);    \
    else if (w2f) launch(f32_conv2_fwd_kernel<T, false, false, false, 2, true>, 0);  \
    else launch(f32_conv2_fwd_kernel<T, false>, 0);                                  \
    break;
  switch (tpb) {
    C2F_CASE(1)
    C2F_CASE(2)
    C2F_CASE(3)
    C2F_CASE(4)
    C2F_CASE(5)
    C2F_CASE(6)
    default:
      if (ad.nblk > 0) launch(f32_conv2_fwd_kernel<7, true>, ad.nblk);
      else if (fuse1) launch(f32_conv2_fwd_kernel<7, false, true, true>, 0);
      else if (prew) launch(f32_conv2_fwd_kernel<7, false, true>, 0);
      else if (w2f) launch(f32_conv2_fwd_kernel<7, false, false, false, 2, true>, 0);
      else launch(f32_conv2_fwd_kernel<7, false>, 0);
  }
#undef C2F_CASE
}

void f32_fc1_fwd(const at::Tensor& a2, at::Tensor& w3, at::Tensor& zpart, const c10::optional<at::Tensor>& g3,
                 const c10::optional<at::Tensor>& m3, const c10::optional<at::Tensor>& v3,
                 const c10::optional<at::Tensor>& state, double lr, double beta1, double beta2, double eps,
                 double grad_scale, int64_t rule) {
  const int B = a2.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_fc1_fwd: batch 1..128");
  check_f32(a2, (int64_t)B * 3136, "f32_fc1_fwd: a2");
  check_f32(w3, 3136 * 1024, "f32_fc1_fwd: w3");
  check_f32(zpart, (int64_t)F1F_KS * B * 1024, "f32_fc1_fwd: zpart [14][B][1024]");
  const c10::optional<at::Tensor> p3 = g3.has_value() && g3->defined() ? c10::optional<at::Tensor>(w3) : c10::nullopt;
  const F32Adam ad = f32_adam_args(p3, g3, m3, v3, state, lr, beta1, beta2, eps, grad_scale, rule, 1, "f32_fc1_fwd");
  const int mt = (B + 15) / 16;
  TORCH_CHECK(ad.nblk == 0 || mt <= 7, "f32_fc1_fwd: the fused dense/kernel update needs B <= 112");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  auto launch = [&](auto kern) {
    const int lds = ad.nblk > 0 ? F1F_LDS_ADAM : mt * 16 * F1F_AS * 4;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kern<<<dim3(16, F1F_KS), 512, lds, stream>>>(a2.data_ptr<float>(), w3.data_ptr<float>(), zpart.data_ptr<float>(),
                                                 B, ad);
  };
  // MIHVD_F32_F1F=0 selects the earlier form (whole-tile update, then the MFMAs) for comparison
  const bool v2 = env_knob("MIHVD_F32_F1F", 1) != 0;
  // MIHVD_F32_F1F_SPLIT=1: the plain forward stages the a2 slice in two K halves (SPLIT above)
  const bool split = v2 && ad.nblk == 0 && env_knob("MIHVD_F32_F1F_SPLIT", 0) != 0;
#define F1F_CASE(T)                                                                                 \
  case T:                                                                                           \
    if (ad.nblk > 0) v2 ? launch(f32_fc1_fwd2_kernel<T, true>) : launch(f32_fc1_fwd_kernel<T, true>); \
    else if (split) launch(f32_fc1_fwd2_kernel<T, false, true>);                                     \
    else v2 ? launch(f32_fc1_fwd2_kernel<T, false>) : launch(f32_fc1_fwd_kernel<T, false>);           \
    break;
  switch (mt) {
    F1F_CASE(1)
    F1F_CASE(2)
    F1F_CASE(3)
    F1F_CASE(4)
    F1F_CASE(5)
    F1F_CASE(6)
    F1F_CASE(7)
    default:
      if (split) launch(f32_fc1_fwd2_kernel<8, false, true>);
      else v2 ? launch(f32_fc1_fwd2_kernel<8, false>) : launch(f32_fc1_fwd_kernel<8, false>);
  }
#undef F1F_CASE
}

void f32_head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                      const at::Tensor& labels, const c10::optional<at::Tensor>& rows,
                      const c10::optional<at::Tensor>& state, int64_t seed, double rate, at::Tensor& h, at::Tensor& dz,
                      at::Tensor& dlog, at::Tensor& stats) {
  const int B = h.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_head: batch 1..128");
  check_f32(zpart, (int64_t)F1F_KS * B * 1024, "f32_head: zpart");
  check_f32(b3, 1024, "f32_head: b3");
  check_f32(w4, 10240, "f32_head: w4");
  check_f32(b4, 10, "f32_head: b4");
  check_f32(h, (int64_t)B * 1024, "f32_head: h");
  check_f32(dz, (int64_t)B * 1024, "f32_head: dz");
  check_f32(dlog, (int64_t)B * 10, "f32_head: dlog");
  check_f32(stats, (int64_t)B * 2, "f32_head: stats");
  TORCH_CHECK(labels.dtype() == at::kLong, "f32_head: labels int64");
  const int n_pool = labels.size(0);
  const int* rp = rows_ptr(rows, n_pool, B, "f32_head");
  int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  TORCH_CHECK(rate >= 0.0 && rate < 1.0, "f32_head: dropout rate in [0, 1)");
  const uint32_t thresh = (uint32_t)(rate * 16777216.0);
  const float keep_scale = rate > 0.0 ? (float)(1.0 / (1.0 - rate)) : 1.f;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  f32_head_kernel<<<B, 256, 0, stream>>>(zpart.data_ptr<float>(), b3.data_ptr<float>(), w4.data_ptr<float>(),
                                         b4.data_ptr<float>(), labels.data_ptr<int64_t>(), rp, n_pool, sp,
                                         (uint32_t)seed, thresh, keep_scale, h.data_ptr<float>(), dz.data_ptr<float>(),
                                         dlog.data_ptr<float>(), stats.data_ptr<float>(), B);
}

}  // namespace mihvd
