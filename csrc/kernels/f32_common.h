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

__device__ __forceinline__ float4 mask_f4(float4 v, bool keep) {
  const uint32_t m = keep ? 0xffffffffu : 0u;
  return make_float4(__uint_as_float(__float_as_uint(v.x) & m), __uint_as_float(__float_as_uint(v.y) & m),
                     __uint_as_float(__float_as_uint(v.z) & m), __uint_as_float(__float_as_uint(v.w) & m));
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

}  // namespace mihvd
