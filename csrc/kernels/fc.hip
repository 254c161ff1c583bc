// Dense layers of the MNIST CNN (horovod/tensorflow_mnist.py:64-71):
//   dense   3136 -> 1024 + ReLU + dropout(0.5)   (fc1)
//   dense_1 1024 -> 10 + softmax cross-entropy   (fc2 / "head")
//
// fc1_fwd   : split-K MFMA GEMM (A = activations [B][3136], B = W3 [3136][1024] bf16). The step is
//             weight-bandwidth bound at B = 100, so 16 column tiles x 14 K slices = 224 blocks each
//             stream a disjoint 28 KB slice of W3 and write an fp32 partial slab (no atomics).
// head      : one block per row: sums the slabs, adds bias, ReLU, counter-based dropout, stores h,
//             computes logits / log-sum-exp / loss / dlogits and back-propagates into dz — the whole
//             fc2 forward+backward fused (K9-K11 of SURVEY.md §2.5).
// fc1_bwd   : one launch, four block roles: dgrad (dz·W3^T with the pool/ReLU mask of conv2's
//             output fused -> g2), wgrad (a2^T·dz -> fp32 gradient written straight into the fusion
//             buffer), db3, and dW4/db4.
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>

#include "common.h"

namespace mihvd {

constexpr int FC1_K = 3136, FC1_N = 1024, FC1_KS = 14, FC1_KSL = FC1_K / FC1_KS;  // 224 = 7 K steps
constexpr int FC1_NT = 64;                                                          // columns per block
constexpr int MAXB = 128;                                                           // batch limit (8 M tiles)
constexpr int F1_ASTR = FC1_KSL + 8;   // 232 elements = 464 B rows (16 B aligned)
constexpr int F1_WSTR = FC1_NT + 8;    // 72 elements = 144 B rows (8 B aligned)
constexpr int F1_LDS = (MAXB * F1_ASTR + FC1_KSL * F1_WSTR) * 2;

// grid (16, 14): blockIdx.x = 64-column tile, blockIdx.y = K slice. 256 threads = 4 waves.
__global__ void __launch_bounds__(256) fc1_fwd_kernel(const u16* __restrict__ a2, const u16* __restrict__ w3,
                                                      float* __restrict__ zpart, int B) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  u16* As = smem;                     // [Mpad][F1_ASTR]
  u16* Ws = smem + MAXB * F1_ASTR;    // [224][F1_WSTR]
  const int nt = blockIdx.x, ks = blockIdx.y, t = threadIdx.x;
  const int MT = (B + 15) >> 4, Mpad = MT * 16;
  const int k0 = ks * FC1_KSL;
  for (int i = t; i < Mpad * (FC1_KSL / 8); i += 256) {
    const int m = i / (FC1_KSL / 8), c = i % (FC1_KSL / 8);
    uint4 v = make_uint4(0, 0, 0, 0);
    if (m < B) v = *reinterpret_cast<const uint4*>(a2 + (int64_t)m * FC1_K + k0 + c * 8);
    *reinterpret_cast<uint4*>(As + m * F1_ASTR + c * 8) = v;
  }
  for (int i = t; i < FC1_KSL * (FC1_NT / 8); i += 256) {
    const int k = i >> 3, c = i & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(w3 + (int64_t)(k0 + k) * FC1_N + nt * FC1_NT + c * 8);
    *reinterpret_cast<uint2*>(Ws + k * F1_WSTR + c * 8) = make_uint2(v.x, v.y);
    *reinterpret_cast<uint2*>(Ws + k * F1_WSTR + c * 8 + 4) = make_uint2(v.z, v.w);
  }
  __syncthreads();
  const int lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4, q = lr >> 2, p = lr & 3;
  f32x4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < FC1_KSL / 32; ++kk) {
    const u16* wr = Ws + (kk * 32 + 8 * lg + q) * F1_WSTR + wave * 16 + 4 * p;
    const bf16x8 bfr = frag_tr(wr, wr + 4 * F1_WSTR);
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      if (mt < MT) {
        const bf16x8 a = frag_ld128(As + (mt * 16 + lr) * F1_ASTR + kk * 32 + 8 * lg);
        acc[mt] = mfma16(a, bfr, acc[mt]);
      }
    }
  }
  float* out = zpart + (int64_t)ks * B * FC1_N;
  const int col = nt * FC1_NT + wave * 16 + lr;
#pragma unroll
  for (int mt = 0; mt < 8; ++mt) {
    if (mt < MT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mt * 16 + 4 * lg + i;
        if (m < B) out[(int64_t)m * FC1_N + col] = acc[mt][i];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ //
// head: one block per row b, 256 threads x 4 features.
// ------------------------------------------------------------------------------------------ //
__global__ void __launch_bounds__(256) head_kernel(
    const float* __restrict__ zpart, int nslab, const float* __restrict__ b3, const float* __restrict__ w4,
    const float* __restrict__ b4, const int64_t* __restrict__ labels, const int* __restrict__ rows, int n_pool,
    int64_t* __restrict__ state, uint32_t seed, uint32_t thresh24, float keep_scale, u16* __restrict__ h_out,
    u16* __restrict__ dz_out, float* __restrict__ dlog_out, float* __restrict__ stats, int B) {
  __shared__ float red[4][10];
  __shared__ float dl[10];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int64_t step = state ? state[ST_FWD] : 0;
  const int n0 = t * 4;
  float z[4];
  {
    const float4 bb = *reinterpret_cast<const float4*>(b3 + n0);
    z[0] = bb.x; z[1] = bb.y; z[2] = bb.z; z[3] = bb.w;
  }
  for (int s = 0; s < nslab; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(zpart + ((int64_t)s * B + b) * FC1_N + n0);
    z[0] += v.x; z[1] += v.y; z[2] += v.z; z[3] += v.w;
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
  // logits partials
  float part[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) part[c] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float* wr = w4 + (int64_t)(n0 + i) * 10;
#pragma unroll
    for (int c = 0; c < 10; ++c) part[c] = fmaf(h[i], wr[c], part[c]);
  }
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    const float s = wave_sum(part[c]);
    if (lane == 0) red[wave][c] = s;
  }
  __syncthreads();
  if (t == 0) {
    int row = b;
    if (rows != nullptr) row = rows[(int)((step * (int64_t)B + b) % n_pool)];
    const int y = (int)labels[row];
    float lg[10], mx = -INFINITY;
    int am = 0;
#pragma unroll
    for (int c = 0; c < 10; ++c) {
      lg[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c] + b4[c];
      if (lg[c] > mx) { mx = lg[c]; am = c; }
    }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) se += __expf(lg[c] - mx);
    const float lse = mx + __logf(se);
    const float invB = 1.0f / (float)B;
#pragma unroll
    for (int c = 0; c < 10; ++c) {
      const float pr = __expf(lg[c] - lse);
      const float d = (pr - (c == y ? 1.f : 0.f)) * invB;
      dl[c] = d;
      dlog_out[b * 10 + c] = d;
    }
    stats[b * 2 + 0] = lse - lg[y];
    stats[b * 2 + 1] = (am == y) ? 1.f : 0.f;
    if (b == 0 && state != nullptr) state[ST_OPT] += 1;
  }
  __syncthreads();
  u16 db[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float* wr = w4 + (int64_t)(n0 + i) * 10;
    float g = 0.f;
#pragma unroll
    for (int c = 0; c < 10; ++c) g = fmaf(dl[c], wr[c], g);
    db[i] = f2bf(h[i] > 0.f ? g * keep_scale : 0.f);
  }
  *reinterpret_cast<uint2*>(dz_out + (int64_t)b * FC1_N + n0) =
      make_uint2((uint32_t)db[0] | ((uint32_t)db[1] << 16), (uint32_t)db[2] | ((uint32_t)db[3] << 16));
}

// ------------------------------------------------------------------------------------------ //
// fc1_bwd: roles by blockIdx.x
//   [0, 196)            dgrad: 16 columns j of dA2 = dz·W3^T, 4 waves split K, fused g2 mask
//   [196, 196+784)      wgrad: 64x64 tile of dW3 = a2^T·dz (K = batch, zero padded)
//   next 4              db3
//   next 4              dW4 (256 features each) ; last block: db4
// ------------------------------------------------------------------------------------------ //
constexpr int FB_DGRAD = FC1_K / 16;                   // 196
constexpr int FB_WGRAD = (FC1_K / 64) * (FC1_N / 64);  // 49 * 16 = 784
constexpr int FB_DB3 = 4, FB_DW4 = 4, FB_DB4 = 1;
constexpr int FB_TOTAL = FB_DGRAD + FB_WGRAD + FB_DB3 + FB_DW4 + FB_DB4;
constexpr int FB_TSTR = 64 + 8;                        // 72 elem rows for the wgrad images
constexpr int FB_LDS = 2 * MAXB * FB_TSTR * 2;         // 36 KB

__global__ void __launch_bounds__(256) fc1_bwd_kernel(
    const u16* __restrict__ dz, const u16* __restrict__ w3, const u16* __restrict__ a2, const u16* __restrict__ h,
    const float* __restrict__ dlog, u16* __restrict__ g2, float* __restrict__ gW3, float* __restrict__ gb3,
    float* __restrict__ gW4, float* __restrict__ gb4, int B) {
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  const int q = lr >> 2, p = lr & 3;
  const int MT = (B + 15) >> 4;
  int bid = blockIdx.x;
  if (bid < FB_DGRAD) {
    // ---- dgrad: columns j0..j0+15, wave = K quarter (256 = 8 K steps) --------------------
    const int j0 = bid * 16;
    f32x4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const u16* wrow = w3 + (int64_t)(j0 + lr) * FC1_N + 8 * lg;   // B[k=n][col=j] = W3[j][n]
    for (int kk = 0; kk < 8; ++kk) {
      const int k = wave * 256 + kk * 32;
      const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(wrow + k);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        if (mt < MT) {
          int m = mt * 16 + lr;
          bf16x8 a;
          if (m < B) a = *reinterpret_cast<const bf16x8*>(dz + (int64_t)m * FC1_N + k + 8 * lg);
          else a = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          acc[mt] = mfma16(a, bfr, acc[mt]);
        }
      }
    }
    float* red = reinterpret_cast<float*>(smem);  // [3 waves][8 tiles][4][64]
    if (wave > 0) {
#pragma unroll
      for (int mt = 0; mt < 8; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(((wave - 1) * 8 + mt) * 4 + i) * 64 + lane] = acc[mt][i];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        if (mt >= MT) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float v = acc[mt][i];
#pragma unroll
          for (int w = 0; w < 3; ++w) v += red[((w * 8 + mt) * 4 + i) * 64 + lane];
          const int m = mt * 16 + 4 * lg + i;
          if (m < B) {
            const int64_t o = (int64_t)m * FC1_K + j0 + lr;
            g2[o] = (bf2f(a2[o]) > 0.f) ? f2bf(v) : (u16)0;
          }
        }
      }
    }
    return;
  }
  bid -= FB_DGRAD;
  if (bid < FB_WGRAD) {
    // ---- wgrad: dW3[j0..+64][n0..+64] = sum_b a2[b][j] dz[b][n] ----------------------------
    const int jt = bid >> 4, ntile = bid & 15;
    const int j0 = jt * 64, n0 = ntile * 64;
    u16* Aim = smem;                  // [Kpad][72]  rows b, cols j
    u16* Bim = smem + MAXB * FB_TSTR; // [Kpad][72]  rows b, cols n
    const int Kpad = (B + 31) & ~31;
    for (int i = t; i < Kpad * 8; i += 256) {
      const int r = i >> 3, c = i & 7;
      uint4 va = make_uint4(0, 0, 0, 0), vb = make_uint4(0, 0, 0, 0);
      if (r < B) {
        va = *reinterpret_cast<const uint4*>(a2 + (int64_t)r * FC1_K + j0 + c * 8);
        vb = *reinterpret_cast<const uint4*>(dz + (int64_t)r * FC1_N + n0 + c * 8);
      }
      *reinterpret_cast<uint2*>(Aim + r * FB_TSTR + c * 8) = make_uint2(va.x, va.y);
      *reinterpret_cast<uint2*>(Aim + r * FB_TSTR + c * 8 + 4) = make_uint2(va.z, va.w);
      *reinterpret_cast<uint2*>(Bim + r * FB_TSTR + c * 8) = make_uint2(vb.x, vb.y);
      *reinterpret_cast<uint2*>(Bim + r * FB_TSTR + c * 8 + 4) = make_uint2(vb.z, vb.w);
    }
    __syncthreads();
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;  // wave's 32x32 sub-tile
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < Kpad; k0 += 32) {
      bf16x8 af[2], bfv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const u16* ar = Aim + (k0 + 8 * lg + q) * FB_TSTR + wm + i * 16 + 4 * p;
        af[i] = frag_tr(ar, ar + 4 * FB_TSTR);
        const u16* br = Bim + (k0 + 8 * lg + q) * FB_TSTR + wn + i * 16 + 4 * p;
        bfv[i] = frag_tr(br, br + 4 * FB_TSTR);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfv[j], acc[i][j]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int jrow = j0 + wm + i * 16 + 4 * lg + e;
          const int ncol = n0 + wn + j * 16 + lr;
          gW3[(int64_t)jrow * FC1_N + ncol] = acc[i][j][e];
        }
    return;
  }
  bid -= FB_WGRAD;
  if (bid < FB_DB3) {
    const int n = bid * 256 + t;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += bf2f(dz[(int64_t)b * FC1_N + n]);
    gb3[n] = s;
    return;
  }
  bid -= FB_DB3;
  if (bid < FB_DW4) {
    float* dls = reinterpret_cast<float*>(smem);  // [B][10]
    for (int i = t; i < B * 10; i += 256) dls[i] = dlog[i];
    __syncthreads();
    const int n = bid * 256 + t;
    float s[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) s[c] = 0.f;
    for (int b = 0; b < B; ++b) {
      const float hv = bf2f(h[(int64_t)b * FC1_N + n]);
#pragma unroll
      for (int c = 0; c < 10; ++c) s[c] = fmaf(hv, dls[b * 10 + c], s[c]);
    }
#pragma unroll
    for (int c = 0; c < 10; ++c) gW4[n * 10 + c] = s[c];
    return;
  }
  // db4
  if (t < 10) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dlog[b * 10 + t];
    gb4[t] = s;
  }
}

// ------------------------------------------------------------------------------------------ //
void fc1_fwd(const at::Tensor& a2, const at::Tensor& w3bf, at::Tensor& zpart) {
  const int B = a2.size(0);
  TORCH_CHECK(B >= 1 && B <= MAXB, "fc1_fwd: batch must be in [1, 128] (got ", B, ")");
  TORCH_CHECK(a2.dtype() == at::kBFloat16 && a2.numel() == (int64_t)B * FC1_K && a2.is_contiguous(), "fc1_fwd: a2");
  TORCH_CHECK(w3bf.dtype() == at::kBFloat16 && w3bf.numel() == (int64_t)FC1_K * FC1_N && w3bf.is_contiguous(), "fc1_fwd: w3");
  TORCH_CHECK(zpart.dtype() == at::kFloat && zpart.numel() == (int64_t)FC1_KS * B * FC1_N, "fc1_fwd: zpart [14][B][1024]");
  static bool attr = [] {
    hipFuncSetAttribute((const void*)fc1_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, F1_LDS);
    return true;
  }();
  (void)attr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  fc1_fwd_kernel<<<dim3(FC1_N / FC1_NT, FC1_KS), 256, F1_LDS, stream>>>((const u16*)a2.data_ptr(), (const u16*)w3bf.data_ptr(),
                                                                       zpart.data_ptr<float>(), B);
}

void head_fwd_bwd(const at::Tensor& zpart, const at::Tensor& b3, const at::Tensor& w4, const at::Tensor& b4,
                  const at::Tensor& labels, const c10::optional<at::Tensor>& rows, const c10::optional<at::Tensor>& state,
                  int64_t seed, double rate, at::Tensor& h, at::Tensor& dz, at::Tensor& dlog, at::Tensor& stats) {
  const int B = h.size(0);
  TORCH_CHECK(zpart.dtype() == at::kFloat && zpart.numel() == (int64_t)FC1_KS * B * FC1_N, "head: zpart");
  TORCH_CHECK(b3.numel() == FC1_N && w4.numel() == FC1_N * 10 && b4.numel() == 10 && w4.dtype() == at::kFloat, "head: params");
  TORCH_CHECK(labels.dtype() == at::kLong, "head: labels must be int64");
  TORCH_CHECK(h.dtype() == at::kBFloat16 && h.numel() == (int64_t)B * FC1_N && dz.numel() == h.numel(), "head: h/dz");
  TORCH_CHECK(dlog.numel() == B * 10 && stats.numel() == B * 2, "head: dlog/stats");
  TORCH_CHECK(rate >= 0.0 && rate < 1.0, "head: dropout rate");
  const int* rp = nullptr;
  int n_pool = labels.numel();
  if (rows.has_value() && rows->defined()) rp = rows->data_ptr<int>();
  else TORCH_CHECK(n_pool >= B, "head: labels shorter than the batch");
  int64_t* sp = (state.has_value() && state->defined()) ? state->data_ptr<int64_t>() : nullptr;
  const uint32_t thresh = (uint32_t)(rate * 16777216.0);
  const float keep_scale = (float)(1.0 / (1.0 - rate));
  auto stream = c10::hip::getCurrentHIPStream().stream();
  head_kernel<<<B, 256, 0, stream>>>(zpart.data_ptr<float>(), FC1_KS, b3.data_ptr<float>(), w4.data_ptr<float>(),
                                     b4.data_ptr<float>(), labels.data_ptr<int64_t>(), rp, n_pool, sp, (uint32_t)seed,
                                     thresh, keep_scale, (u16*)h.data_ptr(), (u16*)dz.data_ptr(), dlog.data_ptr<float>(),
                                     stats.data_ptr<float>(), B);
}

void fc1_bwd(const at::Tensor& dz, const at::Tensor& w3bf, const at::Tensor& a2, const at::Tensor& h,
             const at::Tensor& dlog, at::Tensor& g2, at::Tensor& gW3, at::Tensor& gb3, at::Tensor& gW4, at::Tensor& gb4) {
  const int B = dz.size(0);
  TORCH_CHECK(B >= 1 && B <= MAXB, "fc1_bwd: batch");
  TORCH_CHECK(dz.dtype() == at::kBFloat16 && dz.numel() == (int64_t)B * FC1_N, "fc1_bwd: dz");
  TORCH_CHECK(a2.numel() == (int64_t)B * FC1_K && g2.numel() == a2.numel() && g2.dtype() == at::kBFloat16, "fc1_bwd: a2/g2");
  TORCH_CHECK(gW3.numel() == (int64_t)FC1_K * FC1_N && gW3.dtype() == at::kFloat && gW3.is_contiguous(), "fc1_bwd: gW3");
  TORCH_CHECK(gb3.numel() == FC1_N && gW4.numel() == FC1_N * 10 && gb4.numel() == 10, "fc1_bwd: grads");
  static bool attr = [] {
    hipFuncSetAttribute((const void*)fc1_bwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, FB_LDS);
    return true;
  }();
  (void)attr;
  auto stream = c10::hip::getCurrentHIPStream().stream();
  fc1_bwd_kernel<<<FB_TOTAL, 256, FB_LDS, stream>>>((const u16*)dz.data_ptr(), (const u16*)w3bf.data_ptr(),
                                                    (const u16*)a2.data_ptr(), (const u16*)h.data_ptr(),
                                                    dlog.data_ptr<float>(), (u16*)g2.data_ptr(), gW3.data_ptr<float>(),
                                                    gb3.data_ptr<float>(), gW4.data_ptr<float>(), gb4.data_ptr<float>(), B);
}

}  // namespace mihvd
