// Backward convolutions of the MNIST CNN.
//
// conv2_bwd (one launch, three block roles):
//   dgrad  : dA1 = full-correlation of dY2 with W2 (implicit GEMM, K = 25 taps x 64 channels), with
//            the max-pool routing of conv1's output and its ReLU fused into the epilogue -> g1.
//            dY2 is never materialised in HBM: each block expands the pooled gradient g2 through the
//            argmax indices idx2 straight into an LDS image with a zero halo.
//   wgrad  : dW2 per kernel row kh and group of images as an MFMA GEMM over pixels; both operands are
//            read with ds_read_b64_tr_b16 from their natural NHWC images. Each block writes an fp32
//            partial slab (deterministic, no atomics); conv1_wgrad's launch reduces the slabs.
//   misc   : db2 and zeroing of the conv1 gradient (accumulated with atomics next).
// conv1_wgrad (one launch): dW1/db1 from the sparse routed gradient (1 of 4 conv1 outputs per
//   window is non-zero, so it is computed directly on VALU from the pooled gradient) + the dW2 slab
//   reduction into the fusion buffer.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"

namespace mihvd {

constexpr int CB_IPB = 4;                  // images per wgrad block
constexpr int CB_DSTR = 64;                // dgrad dY2 image: pixel stride (elements)
constexpr int CB_DROWS = 11;               // dY2 rows held by a dgrad block
constexpr int CB_DG_LDS = CB_DROWS * 18 * CB_DSTR * 2;          // 25,344 B
constexpr int CB_APIX = 18 * 18 + 6;                             // padded a1 image + zero pixels
constexpr int CB_WSTR = 72;                                      // wgrad dY2 image stride
constexpr int CB_WG_LDS = (CB_APIX * 32 + 224 * CB_WSTR) * 2;    // 53,568 B
constexpr int CB_LDS = CB_WG_LDS > CB_DG_LDS ? CB_WG_LDS : CB_DG_LDS;

__global__ void __launch_bounds__(256) conv2_bwd_kernel(
    const u16* __restrict__ g2, const uint8_t* __restrict__ idx2, const u16* __restrict__ a1,
    const u16* __restrict__ w2bf, u16* __restrict__ g1, float* __restrict__ slab, float* __restrict__ gb2,
    float* __restrict__ gW1, float* __restrict__ gb1, int B, int n_dgrad, int n_wgrad) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  int bid = blockIdx.x;
  if (bid < n_dgrad) {
    // ------------------------------------------------------------------ dgrad (b, half r)
    const int b = bid >> 1, r = bid & 1;
    u16* D = smem;  // [11][18][64]: local row = y' - (7r-2), local col = x' + 2
    for (int i = t; i < CB_DROWS * 18 * CB_DSTR / 8; i += 256) reinterpret_cast<uint4*>(D)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const int ybase = 7 * r - 2;
    for (int i = t; i < 49 * 64; i += 256) {
      const int win = i >> 6, co = i & 63;
      const int64_t gi = (int64_t)b * 3136 + i;
      const u16 g = g2[gi];
      if (g == 0) continue;
      const int d = idx2[gi];
      const int y = 2 * (win / 7) + (d >> 1), x = 2 * (win % 7) + (d & 1);
      const int yl = y - ybase;
      if (yl < 0 || yl >= CB_DROWS) continue;
      D[(yl * 18 + x + 2) * CB_DSTR + co] = g;
    }
    __syncthreads();
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    int pbase[2];
    const int ntl = (wave + 4 < 7) ? 2 : 1;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int m = (wave + 4 * i) * 16 + lr;
      if (m >= 98) m = 0;
      const int yl = m / 14, x = m % 14;
      pbase[i] = ((yl + 4) * 18 + (x + 4)) * CB_DSTR + 8 * lg;
    }
    for (int kk = 0; kk < 25; ++kk) {
      const int kh = kk / 5, kw = kk - kh * 5;
      const int aoff = -(kh * 18 + kw) * CB_DSTR;
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        // B[k = co][n = ci] = W2[kh][kw][ci][co]
        const u16* wp = w2bf + ((int64_t)(kk * 32 + lr) * 64 + ch * 32 + 8 * lg);
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(wp);
        const bf16x8 b1v = *reinterpret_cast<const bf16x8*>(wp + 16 * 64);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (i < ntl) {
            const bf16x8 a = frag_ld128(D + pbase[i] + aoff + ch * 32);
            acc[i][0] = mfma16(a, b0, acc[i][0]);
            acc[i][1] = mfma16(a, b1v, acc[i][1]);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i >= ntl) continue;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = (wave + 4 * i) * 16 + 4 * lg + e;
          if (m >= 98) continue;
          const int y = 7 * r + m / 14, x = m % 14, ci = nt * 16 + lr;
          const int64_t o = (((int64_t)b * 14 + y) * 14 + x) * 32 + ci;
          g1[o] = (bf2f(a1[o]) > 0.f) ? f2bf(acc[i][nt][e]) : (u16)0;
        }
    }
    return;
  }
  bid -= n_dgrad;
  if (bid < n_wgrad) {
    // ------------------------------------------------------------------ wgrad (kh, group)
    const int kh = bid % 5, grp = bid / 5;
    u16* A = smem;                   // [18*18 + 6 zero pixels][32]
    u16* Dm = smem + CB_APIX * 32;   // [224][72]
    f32x4 acc[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int b_end = min(B, (grp + 1) * CB_IPB);
    for (int b = grp * CB_IPB; b < b_end; ++b) {
      __syncthreads();  // previous image fully consumed
      const uint4* src = reinterpret_cast<const uint4*>(a1 + (int64_t)b * 6272);
      for (int i = t; i < CB_APIX * 4; i += 256) {
        const int pix = i >> 2, c = i & 3;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (pix < 324) {
          const int y = pix / 18 - 2, x = pix % 18 - 2;
          if (y >= 0 && y < 14 && x >= 0 && x < 14) v = src[(y * 14 + x) * 4 + c];
        }
        reinterpret_cast<uint4*>(A)[i] = v;
      }
      for (int i = t; i < 224 * CB_WSTR / 8; i += 256) reinterpret_cast<uint4*>(Dm)[i] = make_uint4(0, 0, 0, 0);
      __syncthreads();
      for (int i = t; i < 49 * 64; i += 256) {
        const int win = i >> 6, co = i & 63;
        const int64_t gi = (int64_t)b * 3136 + i;
        const u16 g = g2[gi];
        if (g == 0) continue;
        const int d = idx2[gi];
        const int pix = (2 * (win / 7) + (d >> 1)) * 14 + 2 * (win % 7) + (d & 1);
        Dm[pix * CB_WSTR + co] = g;
      }
      __syncthreads();
      for (int k0 = 0; k0 < 224; k0 += 32) {
        int poff[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int pix = k0 + 8 * lg + q + 4 * h;
          if (pix < 196) {
            const int y = pix / 14, x = pix % 14;
            poff[h] = ((y + kh) * 18 + x) * 32;
          } else {
            poff[h] = 324 * 32;  // zero pixels (6 of them cover +kw*32 + ci)
          }
        }
        const u16* br = Dm + (k0 + 8 * lg + q) * CB_WSTR + wave * 16 + 4 * p;
        const bf16x8 bfr = frag_tr(br, br + 4 * CB_WSTR);
#pragma unroll
        for (int mt = 0; mt < 10; ++mt) {
          const int kw = mt >> 1, ci0 = (mt & 1) * 16;
          const int add = (poff[0] == 324 * 32 ? 0 : kw * 32) + ci0 + 4 * p;
          const int add1 = (poff[1] == 324 * 32 ? 0 : kw * 32) + ci0 + 4 * p;
          const bf16x8 a = frag_tr(A + poff[0] + add, A + poff[1] + add1);
          acc[mt] = mfma16(a, bfr, acc[mt]);
        }
      }
    }
    float* out = slab + (int64_t)grp * 51200;
#pragma unroll
    for (int mt = 0; mt < 10; ++mt) {
      const int kw = mt >> 1, ci0 = (mt & 1) * 16;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ci = ci0 + 4 * lg + e, co = wave * 16 + lr;
        out[((kh * 5 + kw) * 32 + ci) * 64 + co] = acc[mt][e];
      }
    }
    return;
  }
  // ------------------------------------------------------------------ db2 + zero conv1 grads
  float* red = reinterpret_cast<float*>(smem);
  {
    const int co = t & 63, part = t >> 6;
    float s = 0.f;
    for (int row = part; row < B * 49; row += 4) s += bf2f(g2[(int64_t)row * 64 + co]);
    red[part * 64 + co] = s;
  }
  for (int i = t; i < 800; i += 256) gW1[i] = 0.f;
  if (t < 32) gb1[t] = 0.f;
  __syncthreads();
  if (t < 64) gb2[t] = red[t] + red[64 + t] + red[128 + t] + red[192 + t];
}

// ------------------------------------------------------------------------------------------ //
// conv1_wgrad: blocks [0, B): one image each -> atomics into gW1/gb1; blocks [B, B+50): dW2 slabs.
// ------------------------------------------------------------------------------------------ //
__global__ void __launch_bounds__(256) conv1_wgrad_kernel(
    const float* __restrict__ x, const int* __restrict__ rows, int n_pool, const int64_t* __restrict__ state,
    const u16* __restrict__ g1, const uint8_t* __restrict__ idx1, const float* __restrict__ slab, int nslab,
    float* __restrict__ gW1, float* __restrict__ gb1, float* __restrict__ gW2, int B) {
  __shared__ float img[32][33];
  __shared__ float red[8][26][32];
  const int t = threadIdx.x;
  if ((int)blockIdx.x >= B) {
    const int i = ((int)blockIdx.x - B) * 256 + t;  // float4 index, 12800 total
    if (i < 51200 / 4) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int g = 0; g < nslab; ++g) {
        const float4 v = reinterpret_cast<const float4*>(slab + (int64_t)g * 51200)[i];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      reinterpret_cast<float4*>(gW2)[i] = s;
    }
    return;
  }
  const int b = blockIdx.x;
  int row = b;
  if (rows != nullptr) {
    const int64_t step = state ? state[ST_FWD] : 0;
    row = rows[(int)((step * (int64_t)B + b) % n_pool)];
  }
  const float* xi = x + (int64_t)row * 784;
  for (int i = t; i < 32 * 32; i += 256) {
    const int r = i >> 5, c = i & 31;
    const int gy = r - 2, gx = c - 2;
    img[r][c] = (gy >= 0 && gy < 28 && gx >= 0 && gx < 28) ? xi[gy * 28 + gx] : 0.f;
  }
  __syncthreads();
  const int co = t & 31, grp = t >> 5;
  float acc[25], accb = 0.f;
#pragma unroll
  for (int k = 0; k < 25; ++k) acc[k] = 0.f;
  for (int pos = grp; pos < 196; pos += 8) {
    const int64_t o = (int64_t)b * 6272 + pos * 32 + co;
    const float g = bf2f(g1[o]);
    if (g == 0.f) continue;
    const int d = idx1[o];
    const int py = pos / 14, px = pos - py * 14;
    const int y = 2 * py + (d >> 1), xx = 2 * px + (d & 1);
    accb += g;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) acc[kh * 5 + kw] = fmaf(g, img[y + kh][xx + kw], acc[kh * 5 + kw]);
  }
#pragma unroll
  for (int k = 0; k < 25; ++k) red[grp][k][co] = acc[k];
  red[grp][25][co] = accb;
  __syncthreads();
  for (int i = t; i < 26 * 32; i += 256) {
    const int k = i >> 5, c = i & 31;
    float s = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) s += red[g][k][c];
    if (k < 25) atomicAdd(gW1 + k * 32 + c, s);
    else atomicAdd(gb1 + c, s);
  }
}

// ------------------------------------------------------------------------------------------ //
int64_t conv2_wgrad_groups(int64_t B) { return (B + CB_IPB - 1) / CB_IPB; }

void conv2_bwd(const at::Tensor& g2, const at::Tensor& idx2, const at::Tensor& a1, const at::Tensor& w2bf, at::Tensor& g1,
               at::Tensor& slab, at::Tensor& gb2, at::Tensor& gW1, at::Tensor& gb1) {
  const int B = a1.size(0);
  const int G = (int)conv2_wgrad_groups(B);
  TORCH_CHECK(g2.dtype() == at::kBFloat16 && g2.numel() == (int64_t)B * 3136 && idx2.numel() == g2.numel(), "conv2_bwd: g2/idx2");
  TORCH_CHECK(a1.dtype() == at::kBFloat16 && a1.numel() == (int64_t)B * 6272 && g1.numel() == a1.numel(), "conv2_bwd: a1/g1");
  TORCH_CHECK(w2bf.dtype() == at::kBFloat16 && w2bf.numel() == 51200, "conv2_bwd: w2");
  TORCH_CHECK(slab.dtype() == at::kFloat && slab.numel() >= (int64_t)G * 51200, "conv2_bwd: slab must hold ceil(B/4) x 51200");
  TORCH_CHECK(gb2.numel() == 64 && gW1.numel() == 800 && gb1.numel() == 32, "conv2_bwd: grads");
  static bool attr = [] {
    hipFuncSetAttribute((const void*)conv2_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, CB_LDS);
    return true;
  }();
  (void)attr;
  const int n_dgrad = 2 * B, n_wgrad = 5 * G;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  conv2_bwd_kernel<<<n_dgrad + n_wgrad + 1, 256, CB_LDS, stream>>>(
      (const u16*)g2.data_ptr(), idx2.data_ptr<uint8_t>(), (const u16*)a1.data_ptr(), (const u16*)w2bf.data_ptr(),
      (u16*)g1.data_ptr(), slab.data_ptr<float>(), gb2.data_ptr<float>(), gW1.data_ptr<float>(), gb1.data_ptr<float>(), B,
      n_dgrad, n_wgrad);
}

void conv1_wgrad(const at::Tensor& x, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                 const at::Tensor& g1, const at::Tensor& idx1, const at::Tensor& slab, at::Tensor& gW1, at::Tensor& gb1,
                 at::Tensor& gW2) {
  const int B = g1.size(0);
  const int G = (int)conv2_wgrad_groups(B);
  TORCH_CHECK(x.dtype() == at::kFloat && x.size(-1) == 784, "conv1_wgrad: x");
  TORCH_CHECK(g1.numel() == (int64_t)B * 6272 && idx1.numel() == g1.numel(), "conv1_wgrad: g1/idx1");
  TORCH_CHECK(slab.numel() >= (int64_t)G * 51200 && gW2.numel() == 51200 && gW2.is_contiguous(), "conv1_wgrad: slab/gW2");
  TORCH_CHECK(gW1.numel() == 800 && gb1.numel() == 32, "conv1_wgrad: gW1/gb1");
  const int* rp = nullptr;
  int n_pool = x.size(0);
  if (rows.has_value() && rows->defined()) rp = rows->data_ptr<int>();
  const int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  conv1_wgrad_kernel<<<B + 50, 256, 0, stream>>>(x.data_ptr<float>(), rp, n_pool, sp, (const u16*)g1.data_ptr(),
                                                 idx1.data_ptr<uint8_t>(), slab.data_ptr<float>(), G, gW1.data_ptr<float>(),
                                                 gb1.data_ptr<float>(), gW2.data_ptr<float>(), B);
}

}  // namespace mihvd
