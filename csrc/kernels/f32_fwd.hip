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
#include "xgmi_role.h"

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

// `coll` (xgmi_role.h): a co-launched xGMI collective on blocks [0, coll.nblk) -- the fp32 plane's
// row gather of the previous step's updated dense/kernel rows, on the CUs beside this latency-bound
// launch (its blocks are small: several share a CU with the role block); coll.nblk = 0: none. The
// conv blocks follow (nblk is a multiple of 8, so their XCD mapping is unchanged).
__global__ void __launch_bounds__(256) f32_conv1_kernel(
    const float* __restrict__ x, const int* __restrict__ rows, int n_pool, const int64_t* __restrict__ state,
    const float* __restrict__ w1, const float* __restrict__ b1, float* __restrict__ a1, uint8_t* __restrict__ idx1,
    int B, const float* __restrict__ w2, float* __restrict__ w2f, CollRole coll, const float* __restrict__ xpre) {
  __shared__ float xim[32 * 32];  // 28 x 28 image with a 2-pixel zero halo
  const int cb = coll.nblk;
  if ((int)blockIdx.x < cb) {
    coll_gather_run(coll, (int)blockIdx.x);
    return;
  }
  const int id = blockIdx.x - cb;
  if (id >= 4 * B) {
    f32_w2_frag_block(id - 4 * B, w2, w2f);
    return;
  }
  // XCD-contiguous (image, quarter) order: XCD x writes the a1 rows of images [B x / 8, B (x + 1) / 8),
  // the images whose conv2_fwd blocks run on XCD x (same mapping there), so conv2_fwd's staging
  // reads hit that XCD's L2 instead of the MALL
  const int L = xcd_contiguous(id, 0, 4 * B);
  f32_conv1_block<false>(L & 3, L >> 2, x, rows, n_pool, state, w1, b1, a1, idx1, B, xim, xpre);
}

// The batch of step state[ST_FWD] gathered from the resident set into xpre [B][784] (and its labels
// into ypre [B]): the start of a chain that every f32_fc1_bwd continues for the next step (its
// small-reduction blocks, f32_bwd.hip f32_prefetch_next), so conv1 reads its images and the head its
// labels with one load. Run whenever the counter, the epoch order or the set change
// outside a step (FusedMNISTTrainer._prime_batch).
__global__ void __launch_bounds__(256) f32_prime_kernel(const float* __restrict__ x, const int64_t* __restrict__ labels,
                                                        const int* __restrict__ rows, int n_pool,
                                                        const int64_t* __restrict__ state, int B,
                                                        float* __restrict__ xpre, int* __restrict__ ypre) {
  const int b = blockIdx.x, t = threadIdx.x;
  const int64_t step = state[ST_FWD];
  const int row = rows[(int)((step * (int64_t)B + b) % n_pool)];
  if (t < 196) reinterpret_cast<float4*>(xpre + (int64_t)b * 784)[t] = reinterpret_cast<const float4*>(x + (int64_t)row * 784)[t];
  if (t == 196) ypre[b] = (int)labels[row];
}

// ------------------------------------------------------------------------------------------ //
// conv2: a1 [B][14][14][32] -> a2 [B][3136] (NHWC flatten of [7][7][64]) + idx2
//
// M = the 49 B pooling windows of the batch x 4 pixels (pool-window-major), in 16-row tiles; block
// b owns tiles [b TPB, (b+1) TPB) (TPB = ceil(tiles / 256): about one block per CU), which span at
// most two images. The a1 rows those tiles read are staged once as rows of the "tall" image (image
// i = tall rows [18 i, 18 i + 18), padded row r = a1 row r - 2, 18 padded columns). Weights stay in
// registers (each wave's B operand, loaded once from the W2 fragment copy or W2 itself), so the
// MFMA loop has no global load and no barrier; only the A chunks come from LDS (one ds_read_b128
// per 4 MFMAs). Epilogue: 2x2 max-pool + argmax + bias + ReLU in registers.
constexpr int C2F_MAXR = 22;  // tall rows a block's tiles can span

// A block barrier that orders LDS only (see lds_barrier in f32_bwd.hip): register prefetches stay
// in flight across it.
__device__ __forceinline__ void c2f_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ------------------------------------------------------------------------------------------ //
// conv2 forward, 512 threads: wave w = co group (w & 3) x ci half (w >> 2), so the two waves sharing
// a SIMD split K
// (25 taps x 16 channels each, 100 W2 floats per lane) and hide each other's LDS and MFMA latency
// instead of one wave per SIMD running the whole 800-deep chain; twice the threads stage the image.
// The two ci halves' accumulators meet in LDS behind the image (a fixed order: half 0 + half 1);
// the pool epilogue of the block's tiles is split between the halves.
// The image of this form: unpadded 32-float pixels in 18-pixel tall rows, each pixel's eight 16-byte
// chunks XOR-permuted by 2 ((row + column) & 3): the ds_read_b128 of every tap, tile and window-row
// wrap then lands its 16-lane groups on 16 distinct slots (scripts/ldssim_conv2.py model: 1.00 LDS
// cycles per group, against 1.42 for the padded 40 x 20 layout of round 4's 4-wave form).
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

typedef __attribute__((address_space(3))) void c2f_lds_void;

// DMA: the tall image staged by LDS-DMA (global_load_lds_dwordx4: LDS slot s of a wave-instruction is
// its base + 16 B x lane, so the XOR swizzle is applied to the SOURCE chunk: slot s holds chunk
// (s & 7) ^ swz; padding chunks read a zero line), the W2 operand loaded right behind it, one barrier
// retiring both: no staging registers, no LDS write pass.
template <int TPB, bool FRAG, int DEPTH = 2, bool DMA = false>
__global__ void __launch_bounds__(512) f32_conv2_fwd8_kernel(const float* __restrict__ a1, const float* __restrict__ w2,
                                                             const float* __restrict__ b2, float* __restrict__ a2,
                                                             uint8_t* __restrict__ idx2, int B,
                                                             const float* __restrict__ w2f,
                                                             const float* __restrict__ zeros) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* img = smf;
  f32x4* xr = reinterpret_cast<f32x4*>(smf + C2F8_IMG / 4);
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  const int wco = wave & 3, c2 = wave >> 2;
  // XCD-contiguous tile ranges: XCD x takes the images whose a1 rows conv1's blocks on XCD x wrote
  const int nblk = (((49 * B + 3) / 4) + TPB - 1) / TPB;
  const int nwin = 49 * B, T0 = xcd_contiguous((int)blockIdx.x, 0, nblk) * TPB;
  const int gw0 = 4 * T0, gw1 = min(4 * (T0 + TPB), nwin) - 1;
  const int b0 = gw0 / 49, b1i = gw1 / 49;
  const int R0 = 18 * b0 + 2 * ((gw0 - 49 * b0) / 7);
  const int R1 = 18 * b1i + 2 * ((gw1 - 49 * b1i) / 7) + 6;
  const int nch = (R1 - R0) * 144;  // 18 pixels x 8 float4 per tall row
  float wb[100];  // this wave's W2 operand (below)
  if constexpr (DMA) {
    const int w64 = 64 * wave;
#pragma unroll
    for (int it = 0; it < C2F8_MAXCH; ++it) {
      const int sl = t + 512 * it;  // LDS slot (16-byte chunk) this lane fills
      const int rr = sl / 144, rem = sl - rr * 144, c = rem >> 3, q = (rem & 7) ^ c2f8_swz(rr, c);
      const int R = R0 + rr, bb = R / 18, y = R - 18 * bb - 2, xx = c - 2;
      const bool in = sl < nch && y >= 0 && y < 14 && xx >= 0 && xx < 14;
      const float* src = in ? a1 + (((int64_t)bb * 14 + y) * 14 + xx) * 32 + q * 4 : zeros;
      __builtin_amdgcn_global_load_lds((const void*)src, (c2f_lds_void*)(img + 4 * (w64 + 512 * it)), 16, 0, 0);
    }
    const float4* fp = reinterpret_cast<const float4*>(w2f) + (c2 * 4 + wco) * 64 + lane;
#pragma unroll
    for (int tap = 0; tap < 25; ++tap) {
      const float4 v = fp[tap * 512];
      wb[4 * tap + 0] = v.x;
      wb[4 * tap + 1] = v.y;
      wb[4 * tap + 2] = v.z;
      wb[4 * tap + 3] = v.w;
    }
    __syncthreads();  // (vmcnt(0)): the image has landed in LDS
  } else {
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
  }  // register-staged form
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

// ------------------------------------------------------------------------------------------ //
// conv2 forward, split-bf16 products (f32_common.h: NPROD part products per 32-deep k chunk on
// v_mfma_f32_16x16x32_bf16). Same tiles, blocks and epilogue as f32_conv2_fwd8_kernel; the k chunk is
// one tap's 32 channels. 8 waves = co half (w & 1: co groups 2 ch, 2 ch + 1, 16 channels each) x tap
// quarter (w >> 1: taps 0-6 | 7-12 | 13-18 | 19-24; the two waves of a SIMD, w and w + 4, hold
// quarters q and q + 2: 13 or 12 taps per SIMD). Every A fragment read from LDS feeds both co groups
// (2 NPROD MFMAs per 3 ds_read_b128). The image is split into its three bf16 planes while it is
// staged ([plane][tall row][col][32 channels]: 64 B per pixel and plane, 16-byte chunk g of a pixel
// at chunk g ^ x9f_swz); the W2 operand of a tap is read from the forward fragment copy and split in
// registers one tap ahead; the tap loop is tap-outer, tile-inner (one tap's fragments, every tile's
// accumulators). The four quarter partials of a tile meet in LDS (over the dead image) and quarter
// u % 4 finishes tile u, summing q0 + q1 + q2 + q3 in that order.
constexpr int X9F_PS = 16;                              // dwords per pixel and plane
constexpr int X9F_PLANE = C2F_MAXR * 18 * X9F_PS;       // dwords per plane
constexpr int X9F_IMG = 3 * X9F_PLANE * 4;              // 76,032 B
constexpr int x9f_lds(int tpb) {                       // the image, or the exchange if larger
  return X9F_IMG > 4 * 2 * 2 * tpb * 64 * 16 ? X9F_IMG : 4 * 2 * 2 * tpb * 64 * 16;
}
__device__ __forceinline__ int x9f_swz(int r, int x) { return (((x >> 1) + (r >> 1)) & 1) << 1; }

template <int TPB, int NPROD>
__global__ void __launch_bounds__(512) f32x9_conv2_fwd_kernel(const float* __restrict__ a1, const float* __restrict__ w2f,
                                                              const float* __restrict__ b2, float* __restrict__ a2,
                                                              uint8_t* __restrict__ idx2, int B) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  uint32_t* img = reinterpret_cast<uint32_t*>(smf);
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, g = lane >> 4;
  const int ch = wave & 1, q = wave >> 1;  // co half, tap quarter
  const int tap0 = q == 0 ? 0 : 6 * q + 1, ntap = q == 0 ? 7 : 6;
  const int nblk = (((49 * B + 3) / 4) + TPB - 1) / TPB;
  const int nwin = 49 * B, T0 = xcd_contiguous((int)blockIdx.x, 0, nblk) * TPB;
  const int gw0 = 4 * T0, gw1 = min(4 * (T0 + TPB), nwin) - 1;
  const int b0 = gw0 / 49, b1i = gw1 / 49;
  const int R0 = 18 * b0 + 2 * ((gw0 - 49 * b0) / 7);
  const int R1 = 18 * b1i + 2 * ((gw1 - 49 * b1i) / 7) + 6;
  const int nch = (R1 - R0) * 144;  // 18 pixels x 8 float4 per tall row
  // W2 operand of a tap and co group cg: W2[tap][8 g + j][16 cg + lr], j < 8 = two float4 of the
  // fragment copy fwd [tap][c2][cg][lane][j] = W2[tap][16 c2 + 4 lg + j][16 cg + lr]
  // (c2 = g >> 1, lg = 2 (g & 1) + h)
  const float4* wf = reinterpret_cast<const float4*>(w2f) + ((g >> 1) * 4 + 2 * ch) * 64 + lr + 32 * (g & 1);
  float4 wraw[2][2];
  auto load_w = [&](int tap) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      wraw[c][0] = wf[tap * 512 + 64 * c];
      wraw[c][1] = wf[tap * 512 + 64 * c + 16];
    }
  };
  load_w(tap0);
  // stage: a1 chunk (pixel, 4 channels) -> its 4 bf16 in each plane
  {
    float4 iv[C2F8_MAXCH];
#pragma unroll
    for (int it = 0; it < C2F8_MAXCH; ++it) {
      const int i = min(t + 512 * it, nch - 1);
      const int rr = i / 144, rem = i - rr * 144, c = rem >> 3, chn = rem & 7;
      const int R = R0 + rr, bb = R / 18, y = R - 18 * bb - 2, xx = c - 2;
      const bool in = y >= 0 && y < 14 && xx >= 0 && xx < 14;
      const float4 v = *reinterpret_cast<const float4*>(
          a1 + (((int64_t)bb * 14 + (in ? y : 0)) * 14 + (in ? xx : 0)) * 32 + chn * 4);
      iv[it] = mask_f4(v, in);
    }
#pragma unroll
    for (int it = 0; it < C2F8_MAXCH; ++it) {
      const int i = t + 512 * it;
      if (i < nch) {
        const int rr = i / 144, rem = i - rr * 144, c = rem >> 3, qc = rem & 7;
        const int o = (rr * 18 + c) * X9F_PS + 4 * ((qc >> 1) ^ x9f_swz(rr, c)) + 2 * (qc & 1);
        uint2 h, m, l;
        x9_split4(iv[it], h, m, l);
        *reinterpret_cast<uint2*>(img + o) = h;
        *reinterpret_cast<uint2*>(img + X9F_PLANE + o) = m;
        *reinterpret_cast<uint2*>(img + 2 * X9F_PLANE + o) = l;
      }
    }
  }
  // this lane's pixel (tall row, column) of every tile, before the tap offset
  int pr[TPB], px[TPB];
#pragma unroll
  for (int u = 0; u < TPB; ++u) {
    const int m = 16 * (T0 + u) + lr;
    const int gw = min(m >> 2, nwin - 1), d = m & 3;
    const int bb = gw / 49, win = gw - 49 * bb, py = win / 7, pxw = win - 7 * py;
    pr[u] = 18 * bb + 2 * py + (d >> 1) - R0;
    px[u] = 2 * pxw + (d & 1);
  }
  f32x4 acc[2][TPB];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int u = 0; u < TPB; ++u) acc[c][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // the image is complete
  auto load_a = [&](int u, int kh, int kw) {
    const int r = pr[u] + kh, x = px[u] + kw;
    const uint32_t* p = img + (r * 18 + x) * X9F_PS + 4 * (g ^ x9f_swz(r, x));
    X9Frag f;
    f.p[0] = *reinterpret_cast<const bf16x8*>(p);
    f.p[1] = *reinterpret_cast<const bf16x8*>(p + X9F_PLANE);
    f.p[2] = *reinterpret_cast<const bf16x8*>(p + 2 * X9F_PLANE);
    return f;
  };
  // the running sums alternate sign tap by tap (f32_common.h x9_neg: the bf16 MFMA's rounding bias
  // cancels over consecutive taps); after tap s they hold (-1)^s times the partial sum
  for (int s = 0; s < ntap; ++s) {  // wave-uniform
    const int tap = tap0 + s, kh = tap / 5, kw = tap - 5 * kh;
    X9Frag wb0 = x9_split8(wraw[0][0], wraw[0][1]);
    X9Frag wb1 = x9_split8(wraw[1][0], wraw[1][1]);
    if (s & 1) {
      wb0 = x9_neg(wb0);
      wb1 = x9_neg(wb1);
    }
    if (s + 1 < ntap) load_w(tap + 1);
    X9Frag fa = load_a(0, kh, kw);
#pragma unroll
    for (int u = 0; u < TPB; ++u) {
      X9Frag fn;
      if (u + 1 < TPB) fn = load_a(u + 1, kh, kw);
      __builtin_amdgcn_sched_barrier(0);  // the next tile's reads ahead of this tile's MFMAs (pinned)
      acc[0][u] = x9_mma<NPROD>(fa, wb0, acc[0][u]);
      acc[1][u] = x9_mma<NPROD>(fa, wb1, acc[1][u]);
      __builtin_amdgcn_sched_barrier(0);
      if (u + 1 < TPB) fa = fn;
      if (s + 1 < ntap) {
        acc[0][u] = f4neg(acc[0][u]);
        acc[1][u] = f4neg(acc[1][u]);
      }
    }
  }
  if ((ntap - 1) & 1) {  // wave-uniform: back to the partial sum's own sign
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int u = 0; u < TPB; ++u) acc[c][u] = f4neg(acc[c][u]);
  }
  // exchange over the dead image: xr[co half][tile][quarter][co group][lane]
  __syncthreads();
  f32x4* xr = reinterpret_cast<f32x4*>(smf);
#pragma unroll
  for (int u = 0; u < TPB; ++u)
    if ((u & 3) != q)
#pragma unroll
      for (int c = 0; c < 2; ++c) xr[(((ch * TPB + u) * 4 + q) * 2 + c) * 64 + lane] = acc[c][u];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < TPB; ++u) {
    if ((u & 3) != q) continue;
    const int gw = 4 * (T0 + u) + g;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 sum = q == 0 ? acc[c][u] : xr[(((ch * TPB + u) * 4 + 0) * 2 + c) * 64 + lane];
#pragma unroll
      for (int qq = 1; qq < 4; ++qq) sum += qq == q ? acc[c][u] : xr[(((ch * TPB + u) * 4 + qq) * 2 + c) * 64 + lane];
      const int co = 16 * (2 * ch + c) + lr;
      if (gw < nwin) {
        const int bb = gw / 49, win = gw - 49 * bb;
        int best;
        const float m = pool4(sum, best);
        const int64_t oo = (int64_t)bb * 3136 + win * 64 + co;
        a2[oo] = fmaxf(m + b2[co], 0.f);
        idx2[oo] = (uint8_t)best;
      }
    }
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
// LDS rows of the a2 slice for MT sample tiles: 16 MT, plus the rows the last chunk pass of the
// staging spills into (512-chunk passes over 56-chunk rows; those rows are never read)
constexpr int f1f_rows(int mt) { return ((mt * 16 * 56 + 511) / 512) * 512 / 56 + 1; }
constexpr int F1F_LDS = f1f_rows(8) * F1F_AS * 4;  // 119,712 B
static_assert(F1F_LDS <= 163840, "fc1_fwd LDS");

// MFMA core: a wave's NT tiles (sh, sh + 2, ...) are interleaved element-outer, tile-inner, so
// dependent MFMAs sit NT issues apart (16x16x4 f32: 32-cycle issue, 40-cycle dependent latency),
// and the a2 chunks are read from LDS two chunks ahead.
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

template <int MT>
__global__ void __launch_bounds__(512) f32_fc1_fwd2_kernel(const float* __restrict__ a2, const float* __restrict__ w3,
                                                           float* __restrict__ zpart, int B) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  float* As = smf;  // [16 MT][228]: rows = samples, k contiguous
  // XCD-contiguous (K slice, column group) order: the 16 column-group blocks that stage the same a2
  // slice run on one XCD (two slices per XCD), so the slice comes from that XCD's L2 after its first
  // reader instead of being fetched into all eight L2s
  const int L = xcd_contiguous(blockIdx.y * 16 + blockIdx.x, 0, 16 * F1F_KS);
  const int nb = L & 15, ks = L >> 4, t = threadIdx.x;
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
  // The a2 slice's loads, then the 56 W3 loads, then the a2 LDS writes: the writes wait (in-order
  // vmcnt) for the a2 loads alone and the MFMA chain consumes the W3 fragments as they arrive. The
  // raw values are masked only at the store, and every thread stores all PER chunks (the tail's
  // chunks past the slice land in spare LDS rows, see f32_fc1_fwd): a mask right after each load
  // made the compiler wait for the a2 loads before issuing W3, and the tail chunk's load, used only
  // under the store's condition, was sunk behind the W3 loads, whose vmcnt(0) then held the whole
  // block until every W3 fragment had arrived (the MFMA loop never overlapped the W3 stream).
  float4 v[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = min(t + 512 * it, NCH - 1), r = i / 56, cc = i - 56 * r;
    v[it] = *reinterpret_cast<const float4*>(a2 + (int64_t)min(r, B - 1) * 3136 + k0 + 4 * cc);
  }
  __builtin_amdgcn_sched_barrier(0);
  {
    const int64_t wo = (int64_t)(k0 + 4 * lg) * 1024 + n;
#pragma unroll
    for (int q = 0; q < 14; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) wa[4 * q + j] = w3[wo + (16 * q + j) * 1024];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int it = 0; it < PER; ++it) {
      const int i = t + 512 * it, r = i / 56, cc = i - 56 * r;  // r < F1F_ROWS(MT) for every i
      *reinterpret_cast<float4*>(As + r * F1F_AS + 4 * cc) = mask_f4(v[it], r < B);
    }
    // LDS-only barrier: the W3 fragments (issued before the a2 writes, read from HBM) stay in
    // flight; the MFMA chain consumes them in issue order
    c2f_lds_barrier();
    if (sh == 0)
      f1f_mma<NT0, 0, 14>(wa, bp, acc);
    else
      f1f_mma<NT1, 0, 14>(wa, bp, acc);
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
// fc1 forward on split-bf16 products (f32_common.h): the same grid, slices, waves and slab stores as
// f32_fc1_fwd2_kernel; the 224-deep slice is 7 k chunks of 32. A = W3^T: a lane's 8 consecutive k of
// its column n (the same 56 HBM loads per lane), split in registers chunk by chunk; B = a2^T: the
// slice's three bf16 planes staged once per block ([plane][row][240]: the 16-byte reads of a 16-lane
// group hit 16 distinct slots for every chunk), so an A fragment feeds every tile's NPROD MFMAs and
// a B read 3 ds_read_b128. Sign-alternating accumulation as in conv2_fwd. Batches of up to 112 (the
// planes of 7 sample tiles fill the LDS); larger ones take the fp32-input form.
constexpr int X6F1_S = 240;                        // bf16 per plane row
constexpr int x6f1_plane(int mt) { return mt * 16 * X6F1_S / 2; }  // dwords per plane
static_assert(3 * x6f1_plane(7) * 4 <= 163840, "split fc1_fwd planes");

template <int MT, int NPROD>
__global__ void __launch_bounds__(512) f32x_fc1_fwd_kernel(const float* __restrict__ a2, const float* __restrict__ w3,
                                                           float* __restrict__ zpart, int B) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  uint32_t* pl = reinterpret_cast<uint32_t*>(smf);
  constexpr int PL = x6f1_plane(MT);
  const int L = xcd_contiguous(blockIdx.y * 16 + blockIdx.x, 0, 16 * F1F_KS);
  const int nb = L & 15, ks = L >> 4, t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, g = lane >> 4;
  const int k0 = ks * F1F_KSL, nt = wave & 3, sh = wave >> 2;
  const int n = nb * 64 + nt * 16 + lr;
  constexpr int NCH = MT * 16 * 56, PER = (NCH + 511) / 512;
  constexpr int NT0 = (MT + 1) / 2, NT1 = MT / 2;
  // the slice's a2 loads, then the 56 W3 loads (A: wa[8 c + j] = W3[k0 + 32 c + 8 g + j][n])
  float4 v[PER];
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = min(t + 512 * it, NCH - 1), r = i / 56, cc = i - 56 * r;
    v[it] = *reinterpret_cast<const float4*>(a2 + (int64_t)min(r, B - 1) * 3136 + k0 + 4 * cc);
  }
  __builtin_amdgcn_sched_barrier(0);
  float wa[56];
  {
    const int64_t wo = (int64_t)(k0 + 8 * g) * 1024 + n;
#pragma unroll
    for (int c = 0; c < 7; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) wa[8 * c + j] = w3[wo + (32 * c + j) * 1024];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int it = 0; it < PER; ++it) {
    const int i = t + 512 * it;
    if (i < NCH) {
      const int r = i / 56, cc = i - 56 * r;
      uint2 h, m, l;
      x9_split4(mask_f4(v[it], r < B), h, m, l);
      const int o = r * (X6F1_S / 2) + 2 * cc;
      *reinterpret_cast<uint2*>(pl + o) = h;
      *reinterpret_cast<uint2*>(pl + PL + o) = m;
      *reinterpret_cast<uint2*>(pl + 2 * PL + o) = l;
    }
  }
  c2f_lds_barrier();  // LDS only: the W3 loads stay in flight
  const int ntl = sh == 0 ? NT0 : NT1;
  f32x4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto load_b = [&](int u, int c) {
    const uint32_t* p = pl + ((sh + 2 * u) * 16 + lr) * (X6F1_S / 2) + 16 * c + 4 * g;
    X9Frag f;
    f.p[0] = *reinterpret_cast<const bf16x8*>(p);
    f.p[1] = *reinterpret_cast<const bf16x8*>(p + PL);
    f.p[2] = *reinterpret_cast<const bf16x8*>(p + 2 * PL);
    return f;
  };
  auto run = [&](auto ntc) {
    constexpr int NT = decltype(ntc)::value;
#pragma unroll
    for (int c = 0; c < 7; ++c) {
      X9Frag fa = x9_split8(make_float4(wa[8 * c], wa[8 * c + 1], wa[8 * c + 2], wa[8 * c + 3]),
                            make_float4(wa[8 * c + 4], wa[8 * c + 5], wa[8 * c + 6], wa[8 * c + 7]));
      if (c & 1) fa = x9_neg(fa);
      X9Frag fb = load_b(0, c);
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        X9Frag fn;
        if (u + 1 < NT) fn = load_b(u + 1, c);
        __builtin_amdgcn_sched_barrier(0);
        acc[u] = x9_mma<NPROD>(fa, fb, acc[u]);
        __builtin_amdgcn_sched_barrier(0);
        if (u + 1 < NT) fb = fn;
        if (c < 6) acc[u] = f4neg(acc[u]);
      }
    }
  };
  if (sh == 0) run(std::integral_constant<int, NT0>{});
  else run(std::integral_constant<int, NT1>{});
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int tt = sh + 2 * u, m = tt * 16 + lr;
    if (u < ntl && m < B)
      *reinterpret_cast<float4*>(zpart + ((int64_t)ks * B + m) * 1024 + nb * 64 + nt * 16 + 4 * g) =
          make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
  }
}

// ------------------------------------------------------------------------------------------ //
// head: one block per sample b (K9-K11 of SURVEY.md §2.5):
//   z = sum of the 14 slabs + b3; h = dropout(relu(z)); logits = h W4 + b4; softmax-xent;
//   dlogits = (softmax - onehot) / B; dz = (dlogits W4^T) * relu'(z) * dropout mask
// ------------------------------------------------------------------------------------------ //
// One thread per feature: 1024 threads (16 waves) per sample. Every slab load is a coalesced
// 256-byte wave access and the logits are 16 wave sums that meet in LDS in a fixed order
// (deterministic). (A 256-thread form with 4 features per thread measured 4.45 vs 4.38 us and the
// whole step 120.0 vs 119.0 us; removed.)
__global__ void __launch_bounds__(1024) f32_head1k_kernel(
    const float* __restrict__ zpart, const float* __restrict__ b3, const float* __restrict__ w4,
    const float* __restrict__ b4, const int64_t* __restrict__ labels, const int* __restrict__ rows, int n_pool,
    int64_t* __restrict__ state, uint32_t seed, uint32_t thresh24, float keep_scale, float* __restrict__ h_out,
    float* __restrict__ dz_out, float* __restrict__ dlog_out, float* __restrict__ stats, int B,
    float* __restrict__ stats_acc, const int* __restrict__ ypre) {
  __shared__ float red[16][10];
  __shared__ float dl[10];
  const int b = blockIdx.x, n = threadIdx.x, lane = n & 63, wave = __builtin_amdgcn_readfirstlane(n >> 6);
  const int64_t step = state ? state[ST_FWD] : 0;
  // resident set (ypre != nullptr): this step's label was gathered ahead by the previous step's
  // fc1_bwd (or f32_prime_kernel): one load instead of counter -> rows -> label
  float parts[F1F_KS];
#pragma unroll
  for (int s = 0; s < F1F_KS; ++s) parts[s] = zpart[((int64_t)s * B + b) * 1024 + n];
  float w[10];  // W4[n][0..9]: 40 bytes, 8-byte aligned
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const float2 v = reinterpret_cast<const float2*>(w4 + n * 10)[k];
    w[2 * k] = v.x;
    w[2 * k + 1] = v.y;
  }
  const float bias = b3[n];
  int y = 0;
  float bias4 = 0.f;  // b4 of lane c (wave 0), loaded with the other operands instead of behind the barrier
  if (wave == 0) {
    if (ypre != nullptr) {
      y = ypre[b];
    } else {
      int row = b;
      if (rows != nullptr) row = rows[(int)((step * (int64_t)B + b) % n_pool)];
      y = (int)labels[row];
    }
    bias4 = b4[min(lane, 9)];
  }
  float z = bias;
#pragma unroll
  for (int s = 0; s < F1F_KS; ++s) z += parts[s];
  const bool keep = thresh24 == 0 || dropout_keep(seed, (uint32_t)step, (uint32_t)(b * 1024 + n), thresh24);
  const float hv = keep ? fmaxf(z, 0.f) * keep_scale : 0.f;
  h_out[(int64_t)b * 1024 + n] = hv;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    const float sc = wave_sum(hv * w[c]);
    if (lane == 0) red[wave][c] = sc;
  }
  __syncthreads();
  if (wave == 0) {
    const int c = min(lane, 9);
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < 16; q += 2) acc += red[q][c] + red[q + 1][c];
    const float lgt = acc + bias4;
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
      if (stats_acc != nullptr) {  // running per-sample sums (this block is the sample's only writer)
        stats_acc[b * 2 + 0] += lse - ly;
        stats_acc[b * 2 + 1] += (am == y) ? 1.f : 0.f;
      }
      if (b == 0 && state != nullptr) state[ST_OPT] += 1;
    }
  }
  __syncthreads();
  float g = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) g = fmaf(dl[c], w[c], g);
  dz_out[(int64_t)b * 1024 + n] = hv > 0.f ? g * keep_scale : 0.f;
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
                   const c10::optional<at::Tensor>& w2, const c10::optional<at::Tensor>& w2frag, int64_t coll,
                   const c10::optional<at::Tensor>& xpre) {
  const int B = a1.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_conv1_fwd: batch 1..128");
  const CollRole cr = xgmi_role_lookup(coll);
  TORCH_CHECK(cr.nblk % 8 == 0 && (cr.kind == COLL_GATHER || cr.nblk == 0),
              "f32_conv1_fwd: a co-launched collective must be a gather of a multiple of 8 blocks");
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
  const float* xp = nullptr;
  if (xpre.has_value() && xpre->defined()) {
    check_f32(*xpre, (int64_t)B * 784, "f32_conv1_fwd: xpre [B][784]");
    xp = xpre->data_ptr<float>();
  }
  const bool frag = w2.has_value() && w2->defined() && w2frag.has_value() && w2frag->defined();
  if (frag) {
    check_f32(*w2, 51200, "f32_conv1_fwd: w2");
    check_f32(*w2frag, 2 * 51200, "f32_conv1_fwd: w2frag [2][51200]");
  }
  // (100 fragment blocks, one float4 per thread, measured the same: conv1 7.16 us, whole step
  // 117.6-119.1 us either way, profiles/r05/bench_w2f_blocks_ab_r05s.txt)
  f32_conv1_kernel<<<dim3(cr.nblk + 4 * B + (frag ? 4 * W2F_BLOCKS_Y : 0)), 256, 0, stream>>>(
      x.data_ptr<float>(), rp, n_pool, sp, w1.data_ptr<float>(), b1.data_ptr<float>(), a1.data_ptr<float>(),
      idx1.data_ptr<uint8_t>(), B, frag ? w2->data_ptr<float>() : nullptr, frag ? w2frag->data_ptr<float>() : nullptr,
      cr, xp);
}

void f32_prime_batch(const at::Tensor& x, const at::Tensor& labels, const at::Tensor& rows, const at::Tensor& state,
                     at::Tensor& xpre, at::Tensor& ypre) {
  const int B = xpre.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_prime_batch: batch 1..128");
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "f32_prime_batch: x");
  const int n_pool = x.size(0);
  TORCH_CHECK(labels.dtype() == at::kLong && labels.is_contiguous() && labels.size(0) == n_pool, "f32_prime_batch: labels");
  TORCH_CHECK(rows.dtype() == at::kInt && rows.numel() == n_pool, "f32_prime_batch: rows int32 [n_pool]");
  TORCH_CHECK(state.dtype() == at::kLong && state.numel() >= ST_WORDS, "f32_prime_batch: state");
  check_f32(xpre, (int64_t)B * 784, "f32_prime_batch: xpre [B][784]");
  TORCH_CHECK(ypre.dtype() == at::kInt && ypre.numel() == B && ypre.is_contiguous(), "f32_prime_batch: ypre int32 [B]");
  auto stream = c10::hip::getCurrentHIPStream().stream();
  f32_prime_kernel<<<B, 256, 0, stream>>>(x.data_ptr<float>(), labels.data_ptr<int64_t>(), rows.data_ptr<int>(), n_pool,
                                          state.data_ptr<int64_t>(), B, xpre.data_ptr<float>(), ypre.data_ptr<int>());
}

// tiles per block of f32_conv2_fwd for batch B (about one block per CU), and the block count
static int conv2f_tpb(int B) {
  const int nt = (49 * B + 3) / 4;
  return std::min(7, std::max(1, (nt + 255) / 256));
}

// products: 0 = fp32-input MFMAs; 6 / 9 = split-bf16 part products (f32_common.h; needs w2frag)
void f32_conv2_fwd(const at::Tensor& a1, const at::Tensor& w2, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2,
                   const c10::optional<at::Tensor>& w2frag, int64_t products) {
  TORCH_CHECK(products == 0 || products == 6 || products == 9, "f32_conv2_fwd: products 0, 6 or 9");
  const float* w2f = nullptr;
  if (w2frag.has_value() && w2frag->defined()) {
    TORCH_CHECK(w2frag->is_cuda() && w2frag->dtype() == at::kFloat && w2frag->is_contiguous() &&
                    w2frag->numel() >= 51200, "f32_conv2_fwd: w2frag (the forward fragment copy, 51200 floats)");
    w2f = w2frag->data_ptr<float>();
  }
  const int B = a2.size(0);
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_conv2_fwd: batch 1..128");
  check_f32(a1, (int64_t)B * 6272, "f32_conv2_fwd: a1");
  check_f32(w2, 51200, "f32_conv2_fwd: w2");
  check_f32(b2, 64, "f32_conv2_fwd: b2");
  check_f32(a2, (int64_t)B * 3136, "f32_conv2_fwd: a2");
  check_u8(idx2, (int64_t)B * 3136, "f32_conv2_fwd: idx2");
  const int tpb = conv2f_tpb(B), nt = (49 * B + 3) / 4, nblk = (nt + tpb - 1) / tpb;
  TORCH_CHECK(tpb <= 7, "f32_conv2_fwd: at most 7 tiles per block");
  // every block's tall-row span must fit the LDS image (host check of the kernel's assumption)
  for (int blk = 0; blk < nblk; ++blk) {
    const int gw0 = 4 * blk * tpb, gw1 = std::min(4 * (blk + 1) * tpb, 49 * B) - 1;
    const int r0 = 18 * (gw0 / 49) + 2 * ((gw0 % 49) / 7), r1 = 18 * (gw1 / 49) + 2 * ((gw1 % 49) / 7) + 6;
    TORCH_CHECK(r1 - r0 <= C2F_MAXR, "f32_conv2_fwd: row span exceeds the LDS image");
  }
  auto stream = c10::hip::getCurrentHIPStream().stream();
  if (products != 0) {
    TORCH_CHECK(w2f != nullptr, "f32_conv2_fwd: split-bf16 products read the W2 fragment copy (w2frag)");
    auto launch = [&](auto kern, int lds) {
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      kern<<<nblk, 512, lds, stream>>>(a1.data_ptr<float>(), w2f, b2.data_ptr<float>(), a2.data_ptr<float>(),
                                       idx2.data_ptr<uint8_t>(), B);
    };
    const bool p9 = products == 9;
#define X9F_CASE(T)                                                                          \
  case T:                                                                                    \
    if (p9) launch(f32x9_conv2_fwd_kernel<T, 9>, x9f_lds(T));                                \
    else launch(f32x9_conv2_fwd_kernel<T, 6>, x9f_lds(T));                                   \
    break;
    switch (tpb) {
      X9F_CASE(1)
      X9F_CASE(2)
      X9F_CASE(3)
      X9F_CASE(4)
      X9F_CASE(5)
      X9F_CASE(6)
      default:
        X9F_CASE(7)
    }
#undef X9F_CASE
    return;
  }
  // When the grid fits the CUs, request more LDS than the block needs (> half a CU's) so no two
  // blocks share a CU: the dispatcher otherwise doubles blocks up on some CUs while others idle
  // (measured 20.6 -> 19.7 us at B = 100).
  const int lds = nblk <= device_cu_count() ? std::max(C2F8_LDS, 81920 + 1024) : C2F8_LDS;
  // the image staged by LDS-DMA with the W2 fragment copy (r05k: 20.71 -> 19.31 us, whole step
  // 117.42 -> 116.84 us); without the fragment copy (or the zero line) register staging + LDS writes
  const float* zl = w2f != nullptr ? f32_zero_line(stream) : nullptr;
  auto launch = [&](auto kern) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kern<<<nblk, 512, lds, stream>>>(a1.data_ptr<float>(), w2.data_ptr<float>(), b2.data_ptr<float>(),
                                     a2.data_ptr<float>(), idx2.data_ptr<uint8_t>(), B, w2f, zl);
  };
#define C2F8_CASE(T)                                                         \
  case T:                                                                    \
    if (zl) launch(f32_conv2_fwd8_kernel<T, true, 2, true>);                 \
    else if (w2f) launch(f32_conv2_fwd8_kernel<T, true>);                    \
    else launch(f32_conv2_fwd8_kernel<T, false>);                            \
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
}

void f32_fc1_fwd(const at::Tensor& a2, const at::Tensor& w3, at::Tensor& zpart, int64_t products) {
  const int B = a2.size(0);
  TORCH_CHECK(products == 0 || products == 6 || products == 9, "f32_fc1_fwd: products 0, 6 or 9");
  TORCH_CHECK(B >= 1 && B <= F32_MAXB, "f32_fc1_fwd: batch 1..128");
  check_f32(a2, (int64_t)B * 3136, "f32_fc1_fwd: a2");
  check_f32(w3, 3136 * 1024, "f32_fc1_fwd: w3");
  check_f32(zpart, (int64_t)F1F_KS * B * 1024, "f32_fc1_fwd: zpart [14][B][1024]");
  const int mt = (B + 15) / 16;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  if (products != 0 && mt <= 7) {
    auto launchx = [&](auto kern) {
      const int lds = 3 * x6f1_plane(mt) * 4;
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      kern<<<dim3(16, F1F_KS), 512, lds, stream>>>(a2.data_ptr<float>(), w3.data_ptr<float>(),
                                                   zpart.data_ptr<float>(), B);
    };
#define X6F1_CASE(T)                                                       \
  case T:                                                                  \
    if (products == 9) launchx(f32x_fc1_fwd_kernel<T, 9>);                 \
    else launchx(f32x_fc1_fwd_kernel<T, 6>);                               \
    break;
    switch (mt) {
      X6F1_CASE(1)
      X6F1_CASE(2)
      X6F1_CASE(3)
      X6F1_CASE(4)
      X6F1_CASE(5)
      X6F1_CASE(6)
      default:
        X6F1_CASE(7)
    }
#undef X6F1_CASE
    return;
  }
  // (Measured alternatives, removed: the slice staged in two K halves, 10.7 vs 10.4 us; waves split by
  // K half with every W3 fragment loaded by one wave instead of two, 11.20 vs 11.05 us, whole step
  // 116.84 vs 116.91 us, profiles/r05/kbench_f32_r05o.txt -- the second wave's W3 loads hit the cache)
  auto launch = [&](auto kern) {
    const int lds = f1f_rows(mt) * F1F_AS * 4;
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    kern<<<dim3(16, F1F_KS), 512, lds, stream>>>(a2.data_ptr<float>(), w3.data_ptr<float>(), zpart.data_ptr<float>(),
                                                 B);
  };
#define F1F_CASE(T)                          \
  case T:                                    \
    launch(f32_fc1_fwd2_kernel<T>);          \
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
      F1F_CASE(8)
  }
#undef F1F_CASE
}

void f32_head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                      const at::Tensor& labels, const c10::optional<at::Tensor>& rows,
                      const c10::optional<at::Tensor>& state, int64_t seed, double rate, at::Tensor& h, at::Tensor& dz,
                      at::Tensor& dlog, at::Tensor& stats, const c10::optional<at::Tensor>& stats_acc,
                      const c10::optional<at::Tensor>& ypre) {
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
  float* acc = nullptr;
  if (stats_acc.has_value() && stats_acc->defined()) {
    check_f32(*stats_acc, (int64_t)B * 2, "f32_head: stats_acc [B][2]");
    acc = stats_acc->data_ptr<float>();
  }
  TORCH_CHECK(labels.dtype() == at::kLong, "f32_head: labels int64");
  const int n_pool = labels.size(0);
  const int* rp = rows_ptr(rows, n_pool, B, "f32_head");
  int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  // this step's labels gathered ahead (resident set)
  const int* yp = nullptr;
  if (ypre.has_value() && ypre->defined()) {
    TORCH_CHECK(ypre->dtype() == at::kInt && ypre->numel() == B && ypre->is_contiguous(), "f32_head: ypre int32 [B]");
    yp = ypre->data_ptr<int>();
  }
  TORCH_CHECK(rate >= 0.0 && rate < 1.0, "f32_head: dropout rate in [0, 1)");
  const uint32_t thresh = (uint32_t)(rate * 16777216.0);
  const float keep_scale = rate > 0.0 ? (float)(1.0 / (1.0 - rate)) : 1.f;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  f32_head1k_kernel<<<B, 1024, 0, stream>>>(
      zpart.data_ptr<float>(), b3.data_ptr<float>(), w4.data_ptr<float>(), b4.data_ptr<float>(),
      labels.data_ptr<int64_t>(), rp, n_pool, sp, (uint32_t)seed, thresh, keep_scale, h.data_ptr<float>(),
      dz.data_ptr<float>(), dlog.data_ptr<float>(), stats.data_ptr<float>(), B, acc, yp);
}

}  // namespace mihvd
