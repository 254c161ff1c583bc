// Device helpers of the exact-fp32 step (f32_fwd.hip, f32_bwd.hip).
//
// fp32-input MFMAs on gfx950 (cdna_hip_programming.md §3 "FP32-input MFMA"): exact fp32 products,
// fp32 accumulation, 64 FLOP/clk/SIMD (the fp32 vector rate); there is no xf32 fast path.
//   v_mfma_f32_16x16x4_f32: lane l holds A[l & 15][k = l >> 4], B[k = l >> 4][l & 15];
//                           C[row = 4 (l >> 4) + i][col = l & 15]. 32-cycle issue, 40-cycle
//                           dependent latency: keep >= 2 independent accumulators in flight.
//   v_mfma_f32_32x32x2_f32: lane l holds A[l & 31][k = l >> 5], B[k = l >> 5][l & 31];
//                           C[row = (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col = l & 31] (r = 0..15).
//                           64-cycle issue = dependent latency.
#pragma once

#include "common.h"

namespace mihvd {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int F32_MAXB = 128;  // per-GPU batch limit of the fp32 step

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Four 16x16x4 MFMAs over one 16-deep k chunk: lane group g holds k = 4g + j in element j of both
// float4 operands, MFMA j consumes element j.
__device__ __forceinline__ f32x4 mfma4_q(const float4& a, const float4& b, f32x4 c) {
  c = mfma4(a.x, b.x, c);
  c = mfma4(a.y, b.y, c);
  c = mfma4(a.z, b.z, c);
  return mfma4(a.w, b.w, c);
}

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 mask_f4(float4 v, bool keep) {
  const uint32_t m = keep ? 0xffffffffu : 0u;
  return make_float4(__uint_as_float(__float_as_uint(v.x) & m), __uint_as_float(__float_as_uint(v.y) & m),
                     __uint_as_float(__float_as_uint(v.z) & m), __uint_as_float(__float_as_uint(v.w) & m));
}

// XCD-aware order of a role's blocks: the hardware deals a launch's blocks round-robin over the 8
// XCDs (blockIdx & 7), each with its own L2. Returns the logical index of global block g within the
// role's range [lo, hi) such that every XCD gets a contiguous run of logical indices, so blocks that
// read the same data (the 10 wgrad blocks of an image group; conv1's blocks of an image and the conv2_fwd blocks that read its a1 rows) share one XCD's L2 instead of fetching
// it from HBM eight times.
__device__ __forceinline__ int xcd_contiguous(int g, int lo, int hi) {
  const int x = g & 7;
  int before = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int first = lo + ((c - lo) & 7);
    const int cnt = first < hi ? (hi - first + 7) >> 3 : 0;
    if (c < x) before += cnt;
  }
  const int first_x = lo + ((x - lo) & 7);
  return before + ((g - first_x) >> 3);
}

// 2x2 max-pool of one window held in a lane's four accumulator rows (pixels d = 2 dy + dx in scan
// order): the maximum and the index of its FIRST occurrence (the tie rule of TF's MaxPool gradient
// and torch's max_pool2d backward).
__device__ __forceinline__ float pool4(const f32x4& c, int& best) {
  best = 0;
  float m = c[0];
#pragma unroll
  for (int j = 1; j < 4; ++j)
    if (c[j] > m) {
      m = c[j];
      best = j;
    }
  return m;
}

// Adam over a flat fp32 range with no bf16 shadow (the fp32 step's kernels read the fp32
// parameters): the same adam1() as adam_step, so every schedule of the update agrees bit for bit.
struct F32Adam {
  float* p = nullptr;
  const float* g = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  int64_t n4 = 0;              // float4 groups of the range
  const int64_t* state = nullptr;
  float lr = 0.f, b1 = 0.f, b2 = 0.f, eps = 0.f, gscale = 1.f;
  int rule = 0;
  int nblk = 0;                // blocks of the launch that stream this range (0: none)
};

__device__ __forceinline__ AdamCoef f32_adam_coef(const F32Adam& a) {
  return adam_coef((float)a.state[ST_OPT], a.lr, a.b1, a.b2, a.eps, a.gscale, a.rule);
}

__device__ __forceinline__ void adam4_f32(float4& pp, float4& mm, float4& vv, const float4& gg, const AdamCoef& c) {
  adam1(pp.x, mm.x, vv.x, gg.x, c);
  adam1(pp.y, mm.y, vv.y, gg.y, c);
  adam1(pp.z, mm.z, vv.z, gg.z, c);
  adam1(pp.w, mm.w, vv.w, gg.w, c);
}

// Grid-stride stream of the range by blocks [0, a.nblk) of a launch: four float4 of each array
// per lane per round, all 16 loads issued before the first is used (an HBM-latency-bound stream
// needs that many bytes in flight per CU), restrict-qualified locals.
__device__ __forceinline__ void f32_adam_stream(const F32Adam& a, int bid) {
  constexpr int U = 4;
  const AdamCoef c = f32_adam_coef(a);
  float* __restrict__ p = a.p;
  const float* __restrict__ g = a.g;
  float* __restrict__ m = a.m;
  float* __restrict__ v = a.v;
  const int64_t nthr = (int64_t)a.nblk * blockDim.x;
  for (int64_t i0 = (int64_t)bid * blockDim.x + threadIdx.x; i0 < a.n4; i0 += U * nthr) {
    float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = min(i0 + u * nthr, a.n4 - 1);
      pp[u] = reinterpret_cast<const float4*>(p)[i];
      gg[u] = reinterpret_cast<const float4*>(g)[i];
      mm[u] = reinterpret_cast<const float4*>(m)[i];
      vv[u] = reinterpret_cast<const float4*>(v)[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * nthr;
      if (i < a.n4) {
        adam4_f32(pp[u], mm[u], vv[u], gg[u], c);
        reinterpret_cast<float4*>(p)[i] = pp[u];
        reinterpret_cast<float4*>(m)[i] = mm[u];
        reinterpret_cast<float4*>(v)[i] = vv[u];
      }
    }
  }
}


// conv1 of one quarter (q) of image b: x [row][784] fp32 -> a1 [b][14][14][32] + argmax idx1, 25 taps
// in 7 16x16x4 MFMAs (x in LDS, W1 fragments in registers), pool in a lane's 4 accumulators
// (pool-window-major rows). COH: read W1, b1 and the step counter with agent-scope loads (the
// fused form in f32_conv_reduce, whose other blocks update W1/b1 and the counter in the same
// launch; the caller has acquired their release). xim: [32 * 32] floats of LDS.
template <bool COH>
__device__ __forceinline__ float f32_ld(const float* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool COH>
__device__ __forceinline__ void f32_conv1_block(int q, int b, const float* __restrict__ x, const int* __restrict__ rows,
                                                int n_pool, const int64_t* state, const float* w1, const float* b1,
                                                float* __restrict__ a1, uint8_t* __restrict__ idx1, int B, float* xim,
                                                const float* __restrict__ xpre = nullptr) {
  const int t = threadIdx.x;
  const int lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6), lr = lane & 15, lg = lane >> 4;
  // W1 and b1 first, pinned ahead of the image gather (left alone, the scheduler issued them after
  // the image's LDS barrier: a fourth memory round trip behind counter -> rows -> x)
  float wb[2][7];
  int toff[7];
#pragma unroll
  for (int s = 0; s < 7; ++s) {
    const int k = 4 * s + lg, kc = min(k, 24);
    toff[s] = (kc / 5) * 32 + (kc % 5);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) wb[nt][s] = f32_ld<COH>(w1 + kc * 32 + 16 * nt + lr);
  }
  const float bias0 = f32_ld<COH>(b1 + lr), bias1 = f32_ld<COH>(b1 + 16 + lr);
  __builtin_amdgcn_sched_barrier(0);
  // xpre: this step's batch, gathered ahead by the previous step's head (f32_head1k_kernel) or by
  // f32_prime_kernel -- one load instead of the dependent counter -> rows -> image chain
  int row = b;
  if (xpre != nullptr) {
    x = xpre;
  } else if (rows != nullptr) {
    int64_t step = 0;
    if (state) {
      if constexpr (COH) step = __hip_atomic_load(state + ST_FWD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else step = state[ST_FWD];
    }
    row = rows[(int)((step * (int64_t)B + b) % n_pool)];
  }
  const float* xi = x + (int64_t)row * 784;
  float xv[4];
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int i = t + 256 * it, Y = (i >> 5) - 2, X = (i & 31) - 2;
    const bool in = Y >= 0 && Y < 28 && X >= 0 && X < 28;
    xv[it] = mask_f(xi[in ? Y * 28 + X : 0], in);
  }
#pragma unroll
  for (int s = 0; s < 7; ++s)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) wb[nt][s] = mask_f(wb[nt][s], 4 * s + lg < 25);
#pragma unroll
  for (int it = 0; it < 4; ++it) xim[t + 256 * it] = xv[it];
  __syncthreads();
  const int tile_end = min(49, 13 * q + 13);
  for (int tile = 13 * q + wave; tile < tile_end; tile += 4) {  // wave-uniform
    const int wa = 4 * tile + (lr >> 2), d = lr & 3;
    const int pya = wa / 14, pxa = wa - pya * 14;
    const int base = (2 * pya + (d >> 1)) * 32 + 2 * pxa + (d & 1);
    float av[7];
#pragma unroll
    for (int s = 0; s < 7; ++s) av[s] = xim[base + toff[s]];
    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      c0 = mfma4(av[s], wb[0][s], c0);
      c1 = mfma4(av[s], wb[1][s], c1);
    }
    // C[row 4lg + i][col lr] = pixel i of window 4 * tile + lg, channel 16 nt + lr
    const int win = 4 * tile + lg, py = win / 14, px = win - py * 14;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const f32x4 c = nt ? c1 : c0;
      int best;
      const float m = pool4(c, best);
      const int64_t o = (((int64_t)b * 14 + py) * 14 + px) * 32 + 16 * nt + lr;
      a1[o] = fmaxf(m + (nt ? bias1 : bias0), 0.f);
      idx1[o] = (uint8_t)best;
    }
  }
}

// ------------------------------------------------------------------------------------------ //
// Split-bf16 fp32 products. An fp32 value is the EXACT sum of three bf16 parts by round-to-nearest
// (v_cvt_pk_bf16_f32): hi = bf16(x); r = x - hi (exact: |r| <= half a bf16 ulp of x, on x's ulp
// grid: <= 16 significant bits); mid = bf16(r); lo = r - mid, which has at most 8 significant bits,
// so it IS a bf16 value (|mid| <= 2^-8 |x|, |lo| <= 2^-16 |x|). bf16 x bf16 products are exact in
// fp32, and a 16x16x32 bf16 MFMA chain over the part pairs accumulates in fp32:
//   NPROD = 9: all nine pairs -- every product a * b exact, only the fp32 summation order differs
//              from v_mfma_f32_16x16x4_f32 (144 MFMA cycles per 32-deep k chunk instead of 256);
//   NPROD = 6: the pairs down to 2^-16 relative -- the dropped mid*lo, lo*mid, lo*lo are below
//              2^-24 |a b| together (fp32's own rounding unit) and zero-mean under round-to-nearest
//              (96 cycles per chunk: 2.7x the fp32-input MFMA rate).
// Pairs are accumulated smallest first.
// ------------------------------------------------------------------------------------------ //
struct X9Frag {
  bf16x8 p[3];  // hi, mid, lo: 8 consecutive k per lane each
};

__device__ __forceinline__ void x9_split1(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// 4 consecutive-k values -> two dwords (4 bf16) of each plane
__device__ __forceinline__ void x9_split4(const float4& v, uint2& h, uint2& m, uint2& l) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  bf16x4_t hv, mv, lv;
  const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    __bf16 a, b, c;
    x9_split1(e[j], a, b, c);
    hv[j] = a;
    mv[j] = b;
    lv[j] = c;
  }
  h = __builtin_bit_cast(uint2, hv);
  m = __builtin_bit_cast(uint2, mv);
  l = __builtin_bit_cast(uint2, lv);
}

// 8 consecutive-k values (two float4) -> a fragment of each plane
__device__ __forceinline__ X9Frag x9_split8(const float4& a, const float4& b) {
  uint2 h0, m0, l0, h1, m1, l1;
  x9_split4(a, h0, m0, l0);
  x9_split4(b, h1, m1, l1);
  X9Frag f;
  f.p[0] = __builtin_bit_cast(bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
  f.p[1] = __builtin_bit_cast(bf16x8, make_uint4(m0.x, m0.y, m1.x, m1.y));
  f.p[2] = __builtin_bit_cast(bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
  return f;
}

// The bf16 MFMA's internal accumulation is not round-to-nearest: its results are biased toward
// -inf (bench_native/mfma_split_numerics.hip: mean signed error about -0.05 of the rms error per
// output, where v_mfma_f32_16x16x4_f32 is unbiased). Per element that is harmless, but a gradient
// summed over thousands of such outputs with cancellation (db1 / dW1 from conv2_bwd's dA1) picks the
// bias up coherently: 10x the fp32-input MFMA's error. The k loops therefore alternate the sign of
// the running sum chunk by chunk (negate the accumulator and the chunk's B fragment, x9_neg): a
// rounding toward -inf of -(S + X) is a rounding toward +inf of S + X, so consecutive chunks' biases
// cancel.
__device__ __forceinline__ X9Frag x9_neg(const X9Frag& f) {
  X9Frag n;
#pragma unroll
  for (int p = 0; p < 3; ++p) {
    uint4 u = __builtin_bit_cast(uint4, f.p[p]);
    u.x ^= 0x80008000u;
    u.y ^= 0x80008000u;
    u.z ^= 0x80008000u;
    u.w ^= 0x80008000u;
    n.p[p] = __builtin_bit_cast(bf16x8, u);
  }
  return n;
}
__device__ __forceinline__ f32x4 f4neg(const f32x4& c) { return -c; }

// c += A . B over one 32-deep k chunk: the part pairs, smallest first
template <int NPROD>
__device__ __forceinline__ f32x4 x9_mma(const X9Frag& a, const X9Frag& b, f32x4 c) {
  static_assert(NPROD == 6 || NPROD == 9, "6 or 9 part products");
  if constexpr (NPROD == 9) {
    c = mfma16(a.p[2], b.p[2], c);
    c = mfma16(a.p[2], b.p[1], c);
    c = mfma16(a.p[1], b.p[2], c);
  }
  c = mfma16(a.p[2], b.p[0], c);
  c = mfma16(a.p[0], b.p[2], c);
  c = mfma16(a.p[1], b.p[1], c);
  c = mfma16(a.p[1], b.p[0], c);
  c = mfma16(a.p[0], b.p[1], c);
  return mfma16(a.p[0], b.p[0], c);
}

// A 256-byte zero line in device memory (one per device), the source of the padding chunks of
// LDS-DMA staging (global_load_lds cannot mask a lane: a padding lane reads zeros instead). Created
// on the first call outside a stream capture; nullptr while capturing before that (callers then
// use their register-staged form).
inline const float* f32_zero_line(hipStream_t stream) {
  static float* line[64] = {nullptr};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) return nullptr;
  if (line[dev] == nullptr) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(stream, &cs);
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    float* p = nullptr;
    if (hipMalloc(&p, 256) != hipSuccess) return nullptr;
    (void)hipMemset(p, 0, 256);
    line[dev] = p;
  }
  return line[dev];
}

}  // namespace mihvd
