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

namespace mihvd {

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

  const int lane = t & 63, wave = t >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  // This wave's M tiles: wave, wave+4, wave+8, (12 for wave 0). 13 tiles x 16 = 208 >= 196.
  constexpr int MT = 4;
  f32x4 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // Per-lane A row (pixel) of each tile: m = 16*tile + lr -> window = m>>2, d = m&3.
  int abase[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int tile = wave + 4 * i;
    int m = tile * 16 + lr;
    if (m >= 196) m = 0;  // padded rows read a valid pixel; their results are discarded
    const int win = m >> 2, d = m & 3;
    const int y = 2 * (win / 7) + (d >> 1), x = 2 * (win % 7) + (d & 1);
    abase[i] = (y * 18 + x) * 32 + 8 * lg;
  }
  // Every wave computes 4 tiles (tiles 13..15 are dummies on clamped rows, discarded below): no
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
    const int tile = wave + 4 * i;
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

// ------------------------------------------------------------------------------------------ //
void conv1_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
               const at::Tensor& w1, const at::Tensor& b1, at::Tensor& a1, at::Tensor& idx1) {
  const int B = a1.size(0);
  TORCH_CHECK(x.is_cuda() && x.dtype() == at::kFloat && x.is_contiguous() && x.size(-1) == 784, "conv1_fwd: x");
  TORCH_CHECK(a1.dtype() == at::kBFloat16 && a1.numel() == (int64_t)B * 14 * 14 * 32 && a1.is_contiguous(), "conv1_fwd: a1");
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
  TORCH_CHECK(a1.dtype() == at::kBFloat16 && a1.numel() == (int64_t)B * 6272 && a1.is_contiguous(), "conv2_fwd: a1");
  TORCH_CHECK(w2bf.dtype() == at::kBFloat16 && w2bf.numel() == 51200 && w2bf.is_contiguous(), "conv2_fwd: w2 (bf16)");
  TORCH_CHECK(b2.dtype() == at::kFloat && b2.numel() == 64, "conv2_fwd: b2");
  TORCH_CHECK(a2.dtype() == at::kBFloat16 && a2.numel() == (int64_t)B * 3136 && idx2.numel() == a2.numel(), "conv2_fwd: out");
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

}  // namespace mihvd
