// Numerics probe of split-bf16 fp32 dot products on gfx950 (f32_common.h): 16x16 outputs of
// K-long dot products of random fp32 data, formed five ways, each compared with a float64 host
// reference (relative RMS error, mean signed error in units of the reference RMS):
//   f32      v_mfma_f32_16x16x4_f32 chain (the fp32-input MFMA)
//   x9       nine part products per 32-deep chunk, chained through the accumulator
//   x9fresh  nine part products per chunk into a fresh accumulator, chunks added with v_add_f32
//   x6       six part products per chunk, chained
//   hi       the hi parts alone (a bf16 x bf16 product: the scale of the split's parts)
//   x6alt    six part products, chained, the running sum's sign alternated chunk by chunk (the
//            rounding bias of the bf16 MFMA cancels: f32_common.h x9_neg)
// Inputs: uniform [0, 1) or standard normal (mixed signs), K = 800 and 1600.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels bench_native/mfma_split_numerics.hip -o /tmp/msn
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

struct Frag {
  bf16x8 p[3];
};

__device__ __forceinline__ Frag split8(const float* v) {
  Frag f;
  for (int j = 0; j < 8; ++j) {
    const __bf16 h = (__bf16)v[j];
    const float r1 = v[j] - (float)h;
    const __bf16 m = (__bf16)r1;
    const __bf16 l = (__bf16)(r1 - (float)m);
    f.p[0][j] = h;
    f.p[1][j] = m;
    f.p[2][j] = l;
  }
  return f;
}

__device__ __forceinline__ f32x4 mf(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int MODE>
__device__ f32x4 chunk(const Frag& a, const Frag& b, f32x4 c) {
  if constexpr (MODE == 4) return mf(a.p[0], b.p[0], c);  // hi only
  if constexpr (MODE != 3) {  // x9: the three smallest pairs
    c = mf(a.p[2], b.p[2], c);
    c = mf(a.p[2], b.p[1], c);
    c = mf(a.p[1], b.p[2], c);
  }
  c = mf(a.p[2], b.p[0], c);
  c = mf(a.p[0], b.p[2], c);
  c = mf(a.p[1], b.p[1], c);
  c = mf(a.p[1], b.p[0], c);
  c = mf(a.p[0], b.p[1], c);
  return mf(a.p[0], b.p[0], c);
}

// A [16][K], B [K][16] row-major; out [16][16]. One wave.
template <int MODE>
__global__ void dot_kernel(const float* A, const float* B, float* out, int K) {
  const int lane = threadIdx.x, lr = lane & 15, g = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if constexpr (MODE == 0) {
    for (int k0 = 0; k0 < K; k0 += 4)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[lr * K + k0 + g], B[(k0 + g) * 16 + lr], acc, 0, 0, 0);
  } else {
    for (int k0 = 0; k0 < K; k0 += 32) {
      float av[8], bv[8];
      for (int j = 0; j < 8; ++j) {
        av[j] = A[lr * K + k0 + 8 * g + j];
        bv[j] = B[(k0 + 8 * g + j) * 16 + lr];
      }
      const Frag fa = split8(av), fb = split8(bv);
      if constexpr (MODE == 2) {
        acc += chunk<1>(fa, fb, f32x4{0.f, 0.f, 0.f, 0.f});
      } else if constexpr (MODE == 5) {
        Frag nb = fb;
        if ((k0 >> 5) & 1)
          for (int p = 0; p < 3; ++p) nb.p[p] = -nb.p[p];
        acc = chunk<3>(fa, nb, acc);
        if (k0 + 32 < K) acc = -acc;
      } else {
        acc = chunk<MODE>(fa, fb, acc);
      }
    }
  }
  if (MODE == 5 && (((K - 1) >> 5) & 1)) acc = -acc;
  for (int i = 0; i < 4; ++i) out[(4 * g + i) * 16 + lr] = acc[i];
}

int main() {
  const char* names[6] = {"f32", "x9", "x9fresh", "x6", "hi", "x6alt"};
  for (int dist = 0; dist < 2; ++dist)
    for (int K : {800, 1600}) {
      std::mt19937 rng(1234 + K + dist);
      std::uniform_real_distribution<float> U(0.f, 1.f);
      std::normal_distribution<float> N(0.f, 1.f);
      std::vector<float> A(16 * K), B(K * 16);
      for (auto& v : A) v = dist ? N(rng) : U(rng);
      for (auto& v : B) v = N(rng) * 0.05f;
      std::vector<double> ref(256, 0.0);
      for (int m = 0; m < 16; ++m)
        for (int n = 0; n < 16; ++n) {
          double s = 0.0;
          for (int k = 0; k < K; ++k) s += (double)A[m * K + k] * (double)B[k * 16 + n];
          ref[m * 16 + n] = s;
        }
      float *dA, *dB, *dO;
      (void)hipMalloc(&dA, A.size() * 4);
      (void)hipMalloc(&dB, B.size() * 4);
      (void)hipMalloc(&dO, 256 * 4);
      (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
      (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
      double rr = 0.0;
      for (double v : ref) rr += v * v;
      rr = std::sqrt(rr / 256);
      for (int mode = 0; mode < 6; ++mode) {
        switch (mode) {
          case 0: dot_kernel<0><<<1, 64>>>(dA, dB, dO, K); break;
          case 1: dot_kernel<1><<<1, 64>>>(dA, dB, dO, K); break;
          case 2: dot_kernel<2><<<1, 64>>>(dA, dB, dO, K); break;
          case 3: dot_kernel<3><<<1, 64>>>(dA, dB, dO, K); break;
          case 4: dot_kernel<4><<<1, 64>>>(dA, dB, dO, K); break;
          default: dot_kernel<5><<<1, 64>>>(dA, dB, dO, K); break;
        }
        std::vector<float> o(256);
        (void)hipMemcpy(o.data(), dO, 256 * 4, hipMemcpyDeviceToHost);
        double e2 = 0.0, es = 0.0;
        for (int i = 0; i < 256; ++i) {
          const double e = (double)o[i] - ref[i];
          e2 += e * e;
          es += e;
        }
        printf("%s K=%d %-8s rel rms %.3e  mean signed %.3e\n", dist ? "normal " : "uniform", K, names[mode],
               std::sqrt(e2 / 256) / rr, es / 256 / rr);
      }
      (void)hipFree(dA);
      (void)hipFree(dB);
      (void)hipFree(dO);
    }
  return 0;
}
