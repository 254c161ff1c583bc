// Forward convolutions of the MNIST CNN (horovod/tensorflow_mnist.py:49-60), NHWC, SAME padding,
// each with bias + ReLU + 2x2/2 max-pool fused into the epilogue.
//
// conv1 (1 -> 32 channels, K = 25) has too little reduction depth for MFMA: it is a direct VALU
// convolution with the 25 weights of a channel in registers and the image tile (+halo) in LDS.
//
// conv2 (32 -> 64, K = 800) is an implicit GEMM on v_mfma_f32_16x16x32_bf16. The M dimension
// (output pixels) is enumerated *pool-window-major* (m = 4*window + 2*dy + dx), so each 16-row
// MFMA tile holds 4 complete 2x2 windows and a lane's 4 accumulator rows ARE one window of one
// channel: max-pooling, argmax, bias and ReLU happen in registers with no LDS round trip.
// A = the block's image (bf16, [18][18][32] with zero halo, K-contiguous -> ds_read_b128);
// B = the 800x32 weight slice in its natural HWIO layout ([k][co], read with ds_read_b64_tr_b16).
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"
#include "xgmi_role.h"

MIHVD_OPNS_BEGIN

// ------------------------------------------------------------------------------------------ //
// conv1: x[row][784] fp32 -> a1[b][14][14][32] bf16 + argmax idx1 (0..3, u8)
// grid (7, B): blockIdx.x = pair of pooled rows, blockIdx.y = image. 256 threads:
// lane co = t & 31 owns an output channel (25 weights in registers), t >> 5 picks the position.
// ------------------------------------------------------------------------------------------ //
__global__ void __launch_bounds__(256) conv1_fwd_kernel(
    const float* __restrict__ x, const int* __restrict__ rows, int n_pool, const int64_t* __restrict__ state,
    const float* __restrict__ w1, const float* __restrict__ b1, u16* __restrict__ a1, uint8_t* __restrict__ idx1,
    int B) {
  __shared__ float img[8][33];  // 8 input rows (4 conv rows + 2*2 halo) x 32 cols (28 + 2*2)
  const int pr = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  int row = b;
  if (rows != nullptr) {
    const int64_t step = state ? state[ST_FWD] : 0;
    row = rows[(int)((step * (int64_t)B + b) % n_pool)];
  }
  const float* xi = x + (int64_t)row * 784;
  const int co = t & 31, g = t >> 5;
  float w[25];
#pragma unroll
  for (int k = 0; k < 25; ++k) w[k] = w1[k * 32 + co];
  const float bias = b1[co];
  const int y0 = pr * 4 - 2;  // first input row held in LDS
  {
    const int r = t >> 5, c = t & 31;  // 256 threads = 8 rows x 32 cols
    const int gy = y0 + r, gx = c - 2;
    const bool in = gy >= 0 && gy < 28 && gx >= 0 && gx < 28;
    const float v = xi[in ? gy * 28 + gx : 0];
    img[r][c] = mask_f(v, in);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pos = g + 8 * i;  // 0..27: local pooled row pos/14, col pos%14
    if (pos >= 28) break;
    const int pyl = pos / 14, px = pos - pyl * 14;
    float win[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = 0; c < 6; ++c) win[r][c] = img[2 * pyl + r][2 * px + c];
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const float wk = w[kh * 5 + kw];
        s[0] = fmaf(win[kh][kw], wk, s[0]);
        s[1] = fmaf(win[kh][kw + 1], wk, s[1]);
        s[2] = fmaf(win[kh + 1][kw], wk, s[2]);
        s[3] = fmaf(win[kh + 1][kw + 1], wk, s[3]);
      }
    int best = 0;
    float m = s[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
      if (s[j] > m) { m = s[j]; best = j; }
    const float y = fmaxf(m + bias, 0.f);
    const int py = pr * 2 + pyl;
    const int64_t o = (((int64_t)b * 14 + py) * 14 + px) * 32 + co;
    a1[o] = f2bf(y);
    idx1[o] = (uint8_t)best;
  }
}

// ------------------------------------------------------------------------------------------ //
// conv2: a1[b][14][14][32] bf16 -> a2[b][7][7][64] (= [b][3136] NHWC flatten) bf16 + idx2
// grid (2, B): blockIdx.x = 32-channel half of the outputs, blockIdx.y = image. 256 threads.
// ------------------------------------------------------------------------------------------ //
constexpr int C2_IMG = 18 * 18 * 32;     // bf16 elements of the padded input image
constexpr int C2_WROW = 32 + 8;          // weight image row stride (elements): 80 B, 8B aligned
constexpr int C2_W = 800 * C2_WROW;
constexpr int C2_LDS_BYTES = (C2_IMG + C2_W) * 2;

// The conv2 GEMM + pool epilogue of one (image b, 32-channel half) block, from the LDS images,
// with NW waves: wave w owns the M tiles w, w + NW, ... (13 tiles x 16 = 208 >= 196 pixels).
template <int NW = 4>
__device__ __forceinline__ void conv2_core(const u16* img, const u16* wim, const float* __restrict__ b2,
                                           u16* __restrict__ a2, uint8_t* __restrict__ idx2, int half, int b, int t) {
  const int lane = t & 63, wave = t >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int MT = (13 + NW - 1) / NW;
  f32x4 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Per-lane A row (pixel) of each tile: m = 16*tile + lr -> window = m>>2, d = m&3.
  int abase[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int tile = wave + NW * i;
    int m = tile * 16 + lr;
    if (m >= 196) m = 0;  // padded rows read a valid pixel; their results are discarded
    const int win = m >> 2, d = m & 3;
    const int y = 2 * (win / 7) + (d >> 1), x = 2 * (win % 7) + (d & 1);
    abase[i] = (y * 18 + x) * 32 + 8 * lg;
  }
  // Every wave computes MT tiles (tiles 13+ are dummies on clamped rows, discarded below): no
  // runtime guard around an MFMA, which would make hipcc shuttle the accumulators.
  const int q = lr >> 2, p = lr & 3;
  for (int kk = 0; kk < 25; ++kk) {  // (kh, kw): 32 input channels = one K step
    const int kh = kk / 5, kw = kk - kh * 5;
    const int aoff = (kh * 18 + kw) * 32;
    const u16* wr0 = wim + (kk * 32 + 8 * lg + q) * C2_WROW + 4 * p;
    const bf16x8 b0 = frag_tr(wr0, wr0 + 4 * C2_WROW);
    const bf16x8 b1f = frag_tr(wr0 + 16, wr0 + 16 + 4 * C2_WROW);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const bf16x8 a = frag_ld128(img + abase[i] + aoff);
      acc[i][0] = mfma16(a, b0, acc[i][0]);
      acc[i][1] = mfma16(a, b1f, acc[i][1]);
    }
  }
  // Epilogue: lane holds rows 4*lg..4*lg+3 of its tile = one pooling window, column lr.
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int tile = wave + NW * i;
    const int win = tile * 4 + lg;
    if (win >= 49) continue;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const f32x4 c = acc[i][nt];
      int best = 0;
      float m = c[0];
#pragma unroll
      for (int j = 1; j < 4; ++j)
        if (c[j] > m) { m = c[j]; best = j; }
      const int co = half * 32 + nt * 16 + lr;
      const float y = fmaxf(m + b2[co], 0.f);
      const int64_t o = (int64_t)b * 3136 + win * 64 + co;
      a2[o] = f2bf(y);
      idx2[o] = (uint8_t)best;
    }
  }
}

__global__ void __launch_bounds__(256) conv2_fwd_kernel(
    const u16* __restrict__ a1, const u16* __restrict__ w2bf, const float* __restrict__ b2, u16* __restrict__ a2,
    uint8_t* __restrict__ idx2) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  u16* img = smem;            // [18][18][32]
  u16* wim = smem + C2_IMG;   // [800][C2_WROW] (k = (kh*5+kw)*32 + ci, n = co - 32*half)
  const int half = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  // Issue every load first (image: 6 x 16 B, weights: 13 x 16 B per thread), then write LDS.
  const u16* src = a1 + (int64_t)b * 14 * 14 * 32;
  uint4 iv[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int i = min(t + 256 * k, 18 * 18 * 4 - 1);
    const int pix = i >> 2, ch = i & 3;
    const int y = pix / 18 - 2, x = pix % 18 - 2;
    const bool in = y >= 0 && y < 14 && x >= 0 && x < 14;
    const uint4 v = *reinterpret_cast<const uint4*>(src + ((in ? y : 0) * 14 + (in ? x : 0)) * 32 + ch * 8);
    iv[k] = mask_u4(v, in);
  }
  TileLoad<256, 13, 4> lw;
  lw.load(w2bf + half * 32, 64, 800, 800, t);
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int i = t + 256 * k;
    if (i < 18 * 18 * 4) reinterpret_cast<uint4*>(img)[i] = iv[k];
  }
  lw.store(wim, C2_WROW, 800, t);
  __syncthreads();
  conv2_core(img, wim, b2, a2, idx2, half, b, t);
}

// ------------------------------------------------------------------------------------------ //
// conv12: conv1 and conv2 forward in one launch, grid (2, B) like conv2. Each block computes the
// whole conv1 of its image on MFMA — an implicit GEMM M = 784 pixels (pool-window-major), N = 32,
// K = 25 taps zero-padded to one 32-deep MFMA step, bf16 operands from a padded bf16 copy of the
// image in LDS — and writes the pooled activations straight into conv2's LDS input image, so a1
// never makes an HBM round trip on the forward critical path and one launch (and its ramp) is
// gone. The two blocks of an image compute conv1 redundantly (98 MFMAs each) and split the
// global a1/idx1 stores the backward pass needs by channel half.
// ------------------------------------------------------------------------------------------ //
constexpr int C12_XW = 32;                                  // padded bf16 input image: 32 x 32
constexpr int C12_LDS_BYTES = C2_LDS_BYTES + C12_XW * C12_XW * 2;

template <int NW>
__global__ void __launch_bounds__(NW * 64) conv12_fwd_kernel(
    const float* __restrict__ x, const int* __restrict__ rows, int n_pool, const int64_t* __restrict__ state,
    const u16* __restrict__ w1bf, const float* __restrict__ b1, const u16* __restrict__ w2bf,
    const float* __restrict__ b2, u16* __restrict__ a1, uint8_t* __restrict__ idx1, u16* __restrict__ a2,
    uint8_t* __restrict__ idx2, int B, CollRole cr) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  u16* img = smem;                    // [18][18][32] conv2 input (pooled conv1 output + zero halo)
  u16* wim = smem + C2_IMG;           // [800][C2_WROW]
  u16* xim = smem + C2_IMG + C2_W;    // [32][32] bf16 input image, 2-pixel zero halo
  // co-launched xGMI collective (xgmi_role.h) on the first cr.nblk / 2 grid rows (on the CUs the
  // 2 x B image blocks leave idle)
  if ((int)blockIdx.y < (cr.nblk >> 1)) {
    coll_role_run(cr, blockIdx.y * 2 + blockIdx.x);
    return;
  }
  const int half = blockIdx.x, b = blockIdx.y - (cr.nblk >> 1), t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  // 1. loads. The weights do not depend on the data gather, so they are issued first and land
  //    while the dependent chain step -> rows[] -> image runs.
  constexpr int T = NW * 64;
  TileLoad<T, (3200 + T - 1) / T, 4> lw;
  lw.load(w2bf + half * 32, 64, 800, 800, t);
  // B[k][n] = W1[k = kh*5 + kw][n], k >= 25 zero: lane holds k = 8lg + j, n = 16nt + lr
  uint32_t wb[2][4];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const int k0 = 8 * lg + j;
      const uint32_t lo = w1bf[min(k0, 24) * 32 + 16 * nt + lr] & (k0 < 25 ? 0xffffu : 0u);
      const uint32_t hi = w1bf[min(k0 + 1, 24) * 32 + 16 * nt + lr] & (k0 + 1 < 25 ? 0xffffu : 0u);
      wb[nt][j >> 1] = lo | (hi << 16);
    }
  const float bias0 = b1[lr], bias1 = b1[16 + lr];
  int row = b;
  if (rows != nullptr) {
    const int64_t step = state ? state[ST_FWD] : 0;
    row = rows[(int)((step * (int64_t)B + b) % n_pool)];
  }
  const float* xi = x + (int64_t)row * 784;
  float xv[1024 / T];
#pragma unroll
  for (int it = 0; it < 1024 / T; ++it) {
    const int i = t + T * it, Y = (i >> 5) - 2, X = (i & 31) - 2;
    const bool in = Y >= 0 && Y < 28 && X >= 0 && X < 28;
    xv[it] = mask_f(xi[in ? Y * 28 + X : 0], in);
  }
  // 2. LDS: bf16 input image; zero halo ring of conv2's input image (its interior is written by
  //    the conv1 epilogue below)
#pragma unroll
  for (int it = 0; it < (1296 + T - 1) / T; ++it) {
    const int i = t + T * it;
    if (i < 18 * 18 * 4) {
      const int pix = i >> 2, Y = pix / 18, X = pix - Y * 18;
      if (Y < 2 || Y >= 16 || X < 2 || X >= 16) reinterpret_cast<uint4*>(img)[i] = make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int it = 0; it < 1024 / T; ++it) xim[t + T * it] = f2bf(xv[it]);
  // W2 (issued first, landed before the image chain) goes to LDS now, off the conv1 -> conv2 seam
  lw.store(wim, C2_WROW, 800, t);
  __syncthreads();
  // 3. conv1 on MFMA. Lane row m = 16*tile + lr -> window 4*tile + (lr >> 2), pixel d = lr & 3.
  //    Tap offsets of this lane's 8 k values in the padded image (k >= 25 masked to zero).
  int toff[8];
  uint32_t tmask[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = min(8 * lg + j, 24);
    toff[j] = (k / 5) * C12_XW + (k % 5);
    tmask[j] = (8 * lg + j < 25) ? 0xffffu : 0u;
  }
  const bf16x8 bw0 = __builtin_bit_cast(bf16x8, make_uint4(wb[0][0], wb[0][1], wb[0][2], wb[0][3]));
  const bf16x8 bw1 = __builtin_bit_cast(bf16x8, make_uint4(wb[1][0], wb[1][1], wb[1][2], wb[1][3]));
  // The wave's tiles wave + NW*i (i < C1_NT; tile 49+ is a clamped dummy whose results are
  // dropped) go in batches of 4: every LDS gather of a batch is issued before its MFMAs, so the
  // latency is paid once per batch rather than once per tile.
  constexpr int C1_BATCH = 4, C1_NT = (49 + NW - 1) / NW;
#pragma unroll
  for (int i0 = 0; i0 < C1_NT; i0 += C1_BATCH) {
    bf16x8 af[C1_BATCH];
#pragma unroll
    for (int q = 0; q < C1_BATCH; ++q) {
      if (i0 + q < C1_NT) {
        const int tile = min(wave + NW * (i0 + q), 48);
        const int win_a = 4 * tile + (lr >> 2), d = lr & 3;
        const int py_a = win_a / 14, px_a = win_a - py_a * 14;
        const int base = (2 * py_a + (d >> 1)) * C12_XW + 2 * px_a + (d & 1);
        uint32_t av[4];
#pragma unroll
        for (int j = 0; j < 8; j += 2)
          av[j >> 1] = ((uint32_t)xim[base + toff[j]] & tmask[j]) |
                       (((uint32_t)xim[base + toff[j + 1]] & tmask[j + 1]) << 16);
        af[q] = __builtin_bit_cast(bf16x8, make_uint4(av[0], av[1], av[2], av[3]));
      }
    }
    f32x4 cc[C1_BATCH][2];
#pragma unroll
    for (int q = 0; q < C1_BATCH; ++q) {
      if (i0 + q < C1_NT) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        cc[q][0] = mfma16(af[q], bw0, z);
        cc[q][1] = mfma16(af[q], bw1, z);
      }
    }
#pragma unroll
    for (int q = 0; q < C1_BATCH; ++q) {
      const int tile = wave + NW * (i0 + q);
      if (i0 + q >= C1_NT || tile >= 49) continue;
      // C[row 4lg + i][col lr]: window 4*tile + lg, pixel i of its 2x2 window, channel 16nt + lr
      const int win = 4 * tile + lg, py = win / 14, px = win - py * 14;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const f32x4 c = cc[q][nt];
        int best = 0;
        float m = c[0];
#pragma unroll
        for (int j = 1; j < 4; ++j)
          if (c[j] > m) { m = c[j]; best = j; }
        const int co = 16 * nt + lr;
        const u16 yv = f2bf(fmaxf(m + (nt ? bias1 : bias0), 0.f));
        img[((py + 2) * 18 + px + 2) * 32 + co] = yv;
        if (nt == half) {
          const int64_t o = (((int64_t)b * 14 + py) * 14 + px) * 32 + co;
          a1[o] = yv;
          idx1[o] = (uint8_t)best;
        }
      }
    }
  }
  __syncthreads();
  conv2_core<NW>(img, wim, b2, a2, idx2, half, b, t);
}

// ------------------------------------------------------------------------------------------ //
void conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1) {
  const int B = a1.size(0);
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "conv1_fwd: x");
  TORCH_CHECK(a1.dtype() == MIHVD_OP16 && a1.numel() == (int64_t)B * 14 * 14 * 32 && a1.is_contiguous(), "conv1_fwd: a1");
  TORCH_CHECK(idx1.dtype() == at::kByte && idx1.numel() == a1.numel(), "conv1_fwd: idx1");
  TORCH_CHECK(w1.numel() == 800 && b1.numel() == 32 && w1.dtype() == at::kFloat, "conv1_fwd: weights");
  const int* rp = nullptr;
  int n_pool = x.size(0);
  if (rows.has_value() && rows->defined()) {
    TORCH_CHECK(rows->dtype() == at::kInt && rows->numel() == n_pool, "conv1_fwd: rows must be int32 [n_pool]");
    rp = rows->data_ptr<int>();
  } else {
    TORCH_CHECK(n_pool >= B, "conv1_fwd: x has fewer rows than the batch");
  }
  const int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  conv1_fwd_kernel<<<dim3(7, B), 256, 0, stream>>>(x.data_ptr<float>(), rp, n_pool, sp, w1.data_ptr<float>(),
                                                   b1.data_ptr<float>(), (u16*)a1.data_ptr(), idx1.data_ptr<uint8_t>(), B);
}

void conv2_fwd(const at::Tensor& a1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a2, at::Tensor& idx2) {
  const int B = a1.size(0);
  TORCH_CHECK(a1.dtype() == MIHVD_OP16 && a1.numel() == (int64_t)B * 6272 && a1.is_contiguous(), "conv2_fwd: a1");
  TORCH_CHECK(w2bf.dtype() == MIHVD_OP16 && w2bf.numel() == 51200 && w2bf.is_contiguous(), "conv2_fwd: w2 (bf16)");
  TORCH_CHECK(b2.dtype() == at::kFloat && b2.numel() == 64, "conv2_fwd: b2");
  TORCH_CHECK(a2.dtype() == MIHVD_OP16 && a2.numel() == (int64_t)B * 3136 && idx2.numel() == a2.numel(), "conv2_fwd: out");
  static bool attr = [] {
    hipFuncSetAttribute((const void*)conv2_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, C2_LDS_BYTES);
    return true;
  }();
  (void)attr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  conv2_fwd_kernel<<<dim3(2, B), 256, C2_LDS_BYTES, stream>>>((const u16*)a1.data_ptr(), (const u16*)w2bf.data_ptr(),
                                                              b2.data_ptr<float>(), (u16*)a2.data_ptr(),
                                                              idx2.data_ptr<uint8_t>());
}

void conv12_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                const at::Tensor& w1bf, const at::Tensor& b1, const at::Tensor& w2bf, const at::Tensor& b2, at::Tensor& a1,
                at::Tensor& idx1, at::Tensor& a2, at::Tensor& idx2, int64_t coll) {
  const int B = a1.size(0);
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "conv12_fwd: x");
  TORCH_CHECK(a1.dtype() == MIHVD_OP16 && a1.numel() == (int64_t)B * 6272 && a1.is_contiguous(), "conv12_fwd: a1");
  TORCH_CHECK(idx1.dtype() == at::kByte && idx1.numel() == a1.numel(), "conv12_fwd: idx1");
  TORCH_CHECK(w1bf.dtype() == MIHVD_OP16 && w1bf.numel() == 800 && w1bf.is_contiguous(), "conv12_fwd: w1 (bf16)");
  TORCH_CHECK(b1.dtype() == at::kFloat && b1.numel() == 32, "conv12_fwd: b1");
  TORCH_CHECK(w2bf.dtype() == MIHVD_OP16 && w2bf.numel() == 51200 && w2bf.is_contiguous(), "conv12_fwd: w2 (bf16)");
  TORCH_CHECK(b2.dtype() == at::kFloat && b2.numel() == 64, "conv12_fwd: b2");
  TORCH_CHECK(a2.dtype() == MIHVD_OP16 && a2.numel() == (int64_t)B * 3136 && idx2.numel() == a2.numel() &&
                  idx2.dtype() == at::kByte, "conv12_fwd: a2/idx2");
  const int* rp = nullptr;
  int n_pool = x.size(0);
  if (rows.has_value() && rows->defined()) {
    TORCH_CHECK(rows->dtype() == at::kInt && rows->numel() == n_pool, "conv12_fwd: rows must be int32 [n_pool]");
    rp = rows->data_ptr<int>();
  } else {
    TORCH_CHECK(n_pool >= B, "conv12_fwd: x has fewer rows than the batch");
  }
  const int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  static bool attr = [] {
    hipFuncSetAttribute((const void*)conv12_fwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, C12_LDS_BYTES);
    hipFuncSetAttribute((const void*)conv12_fwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, C12_LDS_BYTES);
    return true;
  }();
  (void)attr;
  // 8 waves per block (one block per CU either way, LDS): more waves hide more of the gather/MFMA
  // latency chains than 4
  auto stream = c10::hip::getCurrentHIPStream().stream();
  CollRole cr = xgmi_role_lookup(coll);
  TORCH_CHECK(cr.nblk % 2 == 0, "conv12_fwd: a co-launched collective needs an even number of blocks");
  auto launch = [&](auto kern, int threads) {
    kern<<<dim3(2, B + cr.nblk / 2), threads, C12_LDS_BYTES, stream>>>(
        x.data_ptr<float>(), rp, n_pool, sp, (const u16*)w1bf.data_ptr(), b1.data_ptr<float>(),
        (const u16*)w2bf.data_ptr(), b2.data_ptr<float>(), (u16*)a1.data_ptr(), idx1.data_ptr<uint8_t>(),
        (u16*)a2.data_ptr(), idx2.data_ptr<uint8_t>(), B, cr);
  };
  launch(conv12_fwd_kernel<8>, 512);
}

MIHVD_OPNS_END
