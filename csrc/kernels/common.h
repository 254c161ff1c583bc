// Shared CDNA4 (gfx950) device helpers for the mihvd MNIST hot path.
//
// * wave64 everywhere; MFMA is v_mfma_f32_16x16x32_bf16 (bf16 in, fp32 accumulate).
//   Fragment maps (cdna_hip_programming.md §3): lane l holds
//     A[m = l&15][k = 8*(l>>4) + j], B[k = 8*(l>>4) + j][n = l&15]   (j = 0..7)
//     C[row = 4*(l>>4) + i][col = l&15]                              (i = 0..3)
// * Operand images in LDS come in two shapes:
//     K-contiguous [row][k]  -> one ds_read_b128 per fragment          (frag_kcontig)
//     K-strided    [k][col]  -> two ds_read_b64_tr_b16 per fragment    (frag_tr)
//   so every global tensor is staged in its natural layout and never transposed in HBM.
#pragma once

#include <cstdlib>

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

// The 16-bit operand format. The MFMA kernels (conv_fwd.hip, conv_bwd.hip, fc.hip, w3_tail.h and
// the operand helpers below) are written once against bf16x8 / f2bf / bf2f / mfma16 and compiled
// twice: the default build in namespace mihvd with bf16 operands (v_mfma_f32_16x16x32_bf16), and
// a -DMIHVD_F16 build in namespace mihvd::f16 with IEEE fp16 operands (v_mfma_f32_16x16x32_f16;
// the Keras 'mixed_float16' policy, loss-scaled). Everything else in this header is format-free and
// lives in namespace mihvd for both.
#ifdef MIHVD_F16
#define MIHVD_OPNS_BEGIN namespace mihvd { namespace f16 {
#define MIHVD_OPNS_END } }
#define MIHVD_OP16 at::kHalf
#else
#define MIHVD_OPNS_BEGIN namespace mihvd {
#define MIHVD_OPNS_END }
#define MIHVD_OP16 at::kBFloat16
#endif

namespace mihvd {

typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define LDS_PTR(T) __attribute__((address_space(3))) T*

}  // namespace mihvd

MIHVD_OPNS_BEGIN

#ifdef MIHVD_F16
typedef _Float16 bf16x8 __attribute__((ext_vector_type(8)));  // (the name is the format-free operand vector)
// v_cvt_f16_f32: round-to-nearest-even; past 65504 -> inf, which the loss scaler detects.
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (_Float16)f); }
__device__ __forceinline__ float bf2f(u16 h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
#else
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
// Plain cast: hipcc emits v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserved).
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
#endif

// Fragment from a K-contiguous LDS image: rows are M (or N) indices, k contiguous.
// `p` points at this lane's 8 elements (row r, k0 + 8*(lane>>4)); must be 16-byte aligned.
__device__ __forceinline__ bf16x8 frag_ld128(const u16* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

// Fragment from a K-strided LDS image ([k][col], col contiguous) via two transposed reads.
// rowp0 = address of row (8*(lane>>4) + q) of this k-block, rowp1 = that of row +4, where
// q = (lane&15)>>2, each already offset by the column 4*(lane&3) of the 16-column block.
__device__ __forceinline__ bf16x8 frag_tr(const u16* rowp0, const u16* rowp1) {
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(short4_t))(rowp0));
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(short4_t))(rowp1));
  typedef short short8_t __attribute__((ext_vector_type(8)));
  short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, s);
}

MIHVD_OPNS_END

namespace mihvd {

// Counter-based dropout RNG (stateless: mask(seed, step, index) is recomputable anywhere).
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x7FEB352Du;
  h ^= h >> 15; h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}
// keep with probability 1-rate; rate is quantised to 1/2^24.
__device__ __forceinline__ bool dropout_keep(uint32_t seed, uint32_t step, uint32_t idx, uint32_t thresh24) {
  return (hash3(seed, step, idx) >> 8) >= thresh24;
}

// Sum over the 16 lanes of a DPP row (every lane gets the row's sum): quad xor 1, quad xor 2,
// half-row mirror, row mirror — four v_add_f32 with DPP operands instead of LDS permutes.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// Whole-wave reductions (every lane gets the result): DPP within the four 16-lane rows, then the
// four row results read as scalars — no LDS permutes (ds_bpermute) on the dependency chain.
__device__ __forceinline__ float wave_sum(float v) {
  v = row_sum16(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = row_max16(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// Direct global -> LDS copy of an image of 128-byte rows into the row-XOR-swizzled layout
// lds[row * 64 + 8 * (chunk ^ (row & 7))] (bf16 elements; 8 16-byte chunks per row). One
// global_load_lds_dwordx4 per wave and 64 chunks: the LDS destination of a wave-instruction is
// lane-linear, so the swizzle is applied to the per-lane SOURCE address. No VGPR round trip and no
// ds_write pass; the copy has landed after the next __syncthreads() (its vmcnt(0) covers it).
template <int NT>
__device__ __forceinline__ void glds_swz128(const u16* __restrict__ g, u16* lds, int nchunks, int t) {
  const int lane = t & 63, w0 = (t >> 6) * 64;
  for (int i0 = w0; i0 < nchunks; i0 += NT) {  // wave-uniform bounds
    const int i = i0 + lane, row = i >> 3;
    __builtin_amdgcn_global_load_lds((const void*)(g + row * 64 + 8 * ((i & 7) ^ (row & 7))),
                                     (void __attribute__((address_space(3)))*)(lds + i0 * 8), 16, 0, 0);
  }
}

// Stage a [rows][cpr x 16 B] tile from global (row stride gstride elements) into LDS (row stride
// lstride elements, 16-byte aligned). Rows >= valid_rows are zero-filled. Every load is issued
// before any LDS store and none is predicated (addresses are clamped, the value is selected after),
// so the whole tile costs one memory latency instead of one per iteration.
//
// Split in two phases so several tiles' loads can all be in flight before the first LDS store:
//   TileLoad<NT, MAXIT, CPR> a, w;  a.load(...); w.load(...); a.store(...); w.store(...);
// Out-of-range rows are zeroed with a bit mask, never with a select: hipcc turns a select on a
// loaded value into a branch around the load, which serialises the loads (one wait per load).
template <int NT, int MAXIT, int CPR>
struct TileLoad {
  uint4 v[MAXIT];
  __device__ __forceinline__ void load(const u16* __restrict__ g, int64_t gstride, int rows, int valid_rows, int t) {
    const int total = rows * CPR;
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int i = min(t + it * NT, total - 1);
      const int r = i / CPR, c = i - r * CPR;
      const int rr = min(r, valid_rows - 1);
      const uint32_t mask = (r < valid_rows) ? 0xffffffffu : 0u;
      const uint4 x = *reinterpret_cast<const uint4*>(g + (int64_t)rr * gstride + c * 8);
      v[it] = make_uint4(x.x & mask, x.y & mask, x.z & mask, x.w & mask);
    }
  }
  __device__ __forceinline__ void store(u16* lds, int lstride, int rows, int t) const {
    const int total = rows * CPR;
#pragma unroll
    for (int it = 0; it < MAXIT; ++it) {
      const int i = t + it * NT;
      if (i < total) {
        const int r = i / CPR, c = i - r * CPR;
        *reinterpret_cast<uint4*>(lds + r * lstride + c * 8) = v[it];
      }
    }
  }
};

// Zero a loaded value when `keep` is false without a select (see TileLoad).
__device__ __forceinline__ uint4 mask_u4(uint4 v, bool keep) {
  const uint32_t m = keep ? 0xffffffffu : 0u;
  return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}
__device__ __forceinline__ float mask_f(float v, bool keep) {
  return __uint_as_float(__float_as_uint(v) & (keep ? 0xffffffffu : 0u));
}

}  // namespace mihvd

MIHVD_OPNS_BEGIN

__device__ __forceinline__ uint2 pack4bf(float a, float b, float c, float d) {
  return make_uint2((uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16), (uint32_t)f2bf(c) | ((uint32_t)f2bf(d) << 16));
}

MIHVD_OPNS_END

namespace mihvd {

// Adam update of four consecutive elements (K12 of SURVEY.md §2.5), shared by the flat-buffer
// optimizer (optim.hip) and the dW3 tiles of fc1_wgrad that update W3 straight from the MFMA
// accumulators; both run exactly this code, so the two paths agree bit for bit.
//   rule 0 (TF1, horovod/tensorflow_mnist.py:130): lr_t = lr sqrt(1-b2^t)/(1-b1^t), eps outside
//   rule 1 (torch.optim.Adam): eps added to sqrt(v_hat)
struct AdamCoef {
  float lr_t, eps_t, inv_sqrt_bc2, b1, b2, gscale;
};
__device__ __forceinline__ AdamCoef adam_coef(float t, float lr, float b1, float b2, float eps, float gscale, int rule) {
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  AdamCoef c;
  c.lr_t = rule == 0 ? lr * sqrtf(bc2) / bc1 : lr / bc1;
  c.eps_t = rule == 0 ? eps : eps * sqrtf(bc2);
  c.inv_sqrt_bc2 = rule == 0 ? 1.f : 1.f / sqrtf(bc2);
  c.b1 = b1;
  c.b2 = b2;
  c.gscale = gscale;
  return c;
}
// The step uses the hardware square root and reciprocal (v_sqrt_f32 / v_rcp_f32, 1 ulp) instead of
// the IEEE-rounded sqrtf and division: those expand to ~25 VALU instructions per element (scale,
// div_fmas, fixup, class checks), which made the update VALU-bound wherever it shares CUs with
// compute. The difference is a few ulp of the step (lr-scaled), far below the bf16 shadow's
// resolution; every optimizer kernel runs this same code, so all schedules agree bit for bit.
__device__ __forceinline__ void adam1(float& p, float& m, float& v, const float g, const AdamCoef& c) {
  const float gk = g * c.gscale;
  m = fmaf(c.b1, m, (1.f - c.b1) * gk);
  v = fmaf(c.b2, v, (1.f - c.b2) * gk * gk);
  p -= c.lr_t * m * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(v), c.inv_sqrt_bc2, c.eps_t));
}
}  // namespace mihvd

MIHVD_OPNS_BEGIN

__device__ __forceinline__ uint2 adam4(float4& pp, float4& mm, float4& vv, const float4 gg, const AdamCoef& c) {
  float* pa = &pp.x;
  float* ma = &mm.x;
  float* va = &vv.x;
  const float* ga = &gg.x;
  u16 sh[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    adam1(pa[k], ma[k], va[k], ga[k], c);
    sh[k] = f2bf(pa[k]);
  }
  return make_uint2((uint32_t)sh[0] | ((uint32_t)sh[1] << 16), (uint32_t)sh[2] | ((uint32_t)sh[3] << 16));
}

MIHVD_OPNS_END

namespace mihvd {

// Arguments of an Adam update fused into another kernel (p, m, v, shadow are the slices of the flat
// buffers that the update covers).
struct AdamArgs {
  float* p;
  float* m;
  float* v;
  u16* shadow;
  const int64_t* state;
  float lr, b1, b2, eps, gscale;
  int rule;
};

// CU count of the current device, queried once per device (launch-time grid sizing; a
// hipDeviceGetAttribute per launch costs host time on every step of an eager loop).
// Integer knob from the environment (kernel-study switches read at launch/capture time), or def.
inline int env_knob(const char* name, int def) {
  const char* v = std::getenv(name);
  return (v != nullptr && *v != '\0') ? std::atoi(v) : def;
}

inline int device_cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] == 0) {
    int n = 256;
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    cache[dev] = n > 0 ? n : 256;
  }
  return cache[dev];
}

// Profiling aid (scripts/kbench.py --roles): MIHVD_ROLE_ONLY=<r> makes a launch that packs several
// block roles run only the blocks of role r, so each role can be timed on its own. Unset (the
// normal case) every role runs.
inline int debug_role_only() {
  const char* e = getenv("MIHVD_ROLE_ONLY");
  return e ? atoi(e) : -1;
}

// Profiling aid: MIHVD_DEBUG_EXIT=<phase> makes instrumented kernels return after that phase
// (results are then incomplete), so the cost of each phase can be read off kernel times.
inline int debug_phase_exit() {
  const char* e = getenv("MIHVD_DEBUG_EXIT");
  return e ? atoi(e) : 0;
}

// Step-state words kept on the device so a whole training step replays from a HIP graph:
//   state[0] = forward step index (read by data/dropout kernels, bumped by the optimizer)
//   state[1] = optimizer step t   (bumped by the head kernel, read by the optimizer)
enum { ST_FWD = 0, ST_OPT = 1, ST_WORDS = 4 };

// A memory-streaming Adam update appended to a compute-bound launch (conv2_bwd): after its own
// work every wave of the launch updates the float4 groups w, w + W, w + 2W, ... (256 per group,
// W = waves in the launch) of the flat range [0, 4*n4). Blocks without compute work (on the CUs
// the compute roles leave idle) start at once. Measured on MI355X, the static interleave beats
// work stealing through device-scope atomic counters (per-XCD, one atomic per block and chunk):
// 78.4 vs 79.6 us per step, with no counters to re-arm.
struct AdamTail {
  float* p;
  const float* g;
  float* m;
  float* v;
  u16* shadow;
  int64_t n4;
  const int64_t* state;  // ST_OPT: the optimizer step t
  float lr, b1, b2, eps, gscale;
  int rule;
  int first_free;        // blocks [first_free, grid) have no compute work ...
  int64_t head;          // ... and alone take the chunks [0, head) (64 float4 each) before the shared range
};

}  // namespace mihvd

MIHVD_OPNS_BEGIN

// One float4 of every array per lane per iteration, grid-stride — the loop of the standalone
// adam_kernel (optim.hip), which streams at full HBM rate even on one 4-wave block per CU; the
// arrays are restrict-qualified locals so loads may be hoisted past the previous stores.
__device__ __forceinline__ void adam_tail_stream(const AdamTail& at, const AdamCoef& c, int64_t i, int64_t end,
                                                 int64_t stride) {
  float* __restrict__ p = at.p;
  const float* __restrict__ g = at.g;
  float* __restrict__ m = at.m;
  float* __restrict__ v = at.v;
  u16* __restrict__ sh = at.shadow;
  for (; i < end; i += stride) {
    float4 pp = reinterpret_cast<const float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<const float4*>(m)[i];
    float4 vv = reinterpret_cast<const float4*>(v)[i];
    const uint2 s2 = adam4(pp, mm, vv, gg, c);
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    reinterpret_cast<uint2*>(sh)[i] = s2;
  }
}

// Waves without compute work start at once and run for the whole compute phase, so they take a
// head range of their own (at.head float4 chunks of 64, sized by the caller) before every wave of
// the launch shares the rest. Free waves: every wave of the blocks [first_free, grid), and the
// streamer waves (index >= 8) that blocks of more than 512 threads add to the compute blocks.
__device__ __forceinline__ void adam_tail_run(const AdamTail& at) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int waves = (int)blockDim.x >> 6;
  const int sw = waves - 8 > 0 ? waves - 8 : 0;  // streamer waves per compute block
  const AdamCoef c = adam_coef((float)at.state[ST_OPT], at.lr, at.b1, at.b2, at.eps, at.gscale, at.rule & 0xff);
  const int64_t head4 = min(at.head * 64, at.n4);
  const int n_free = (int)gridDim.x - at.first_free;
  const int64_t nfw = (int64_t)at.first_free * sw + (int64_t)n_free * waves;
  int64_t fw = -1;
  if ((int)blockIdx.x >= at.first_free) fw = (int64_t)at.first_free * sw + (int64_t)((int)blockIdx.x - at.first_free) * waves + wave;
  else if (wave >= 8) fw = (int64_t)blockIdx.x * sw + (wave - 8);
  if (fw >= 0) adam_tail_stream(at, c, fw * 64 + lane, head4, nfw * 64);
  adam_tail_stream(at, c, head4 + ((int64_t)blockIdx.x * waves + wave) * 64 + lane, at.n4, (int64_t)gridDim.x * waves * 64);
}

MIHVD_OPNS_END
