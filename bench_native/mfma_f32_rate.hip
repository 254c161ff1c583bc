// Microbenchmark: sustained v_mfma_f32_16x16x4_f32 / 32x32x2_f32 issue rate on one MI355X, operands
// in registers, NACC independent accumulators per wave, W waves per SIMD (blocks of 4 W waves, one
// block per CU). Calibrates what the fp32 step's kernels can reach (cycles per MFMA per SIMD).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ void __launch_bounds__(1024) mfma16(float* out, int iters, float seed) {
  f32x4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = seed * threadIdx.x, b = seed + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void __launch_bounds__(1024) mfma32(float* out, int iters, float seed) {
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float a = seed * threadIdx.x, b = seed + blockIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static void run(const char* name, K kern, int waves_per_simd, int nacc, int iters, int mfma_flop) {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  const int threads = 256 * waves_per_simd;
  float* out;
  hipMalloc(&out, (size_t)ncu * threads * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  kern<<<ncu, threads>>>(out, iters, 1.0f);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  kern<<<ncu, threads>>>(out, iters, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double per_simd = (double)iters * nacc * waves_per_simd;  // MFMAs per SIMD
  const double flops = per_simd * 4.0 * ncu * mfma_flop;
  const double ghz_ref = clk / 1e6;
  std::printf("%-10s waves/SIMD %d acc %d: %8.3f ms  %7.1f TF/s  %6.1f cycles/MFMA/SIMD at %.2f GHz (max clock)\n", name,
              waves_per_simd, nacc, ms, flops / (ms * 1e-3) / 1e12, ms * 1e-3 * ghz_ref * 1e9 / per_simd, ghz_ref);
  hipFree(out);
}

int main() {
  const int it = 20000;
  run("16x16x4", mfma16<1>, 1, 1, it, 2048);
  run("16x16x4", mfma16<2>, 1, 2, it, 2048);
  run("16x16x4", mfma16<5>, 1, 5, it, 2048);
  run("16x16x4", mfma16<5>, 2, 5, it, 2048);
  run("16x16x4", mfma16<4>, 4, 4, it / 2, 2048);
  run("32x32x2", mfma32<1>, 1, 1, it / 2, 4096);
  run("32x32x2", mfma32<4>, 1, 4, it / 2, 4096);
  run("32x32x2", mfma32<4>, 2, 4, it / 2, 4096);
  return 0;
}
