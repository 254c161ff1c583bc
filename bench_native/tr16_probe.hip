// ds_read_b64_tr_b16 semantics probe (gfx950): LDS holds a [16 rows][32 cols] tile of 16-bit values
// v = 100 * row + col; lane 4q + p of each 16-lane group supplies the address of row q, columns
// 4p .. 4p + 3 (group G of the wave reads rows 4 G .. 4 G + 3). Prints what every lane receives.
//   hipcc --offload-arch=gfx950 -O3 bench_native/tr16_probe.hip -o /tmp/tr16
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void probe(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[16 * 32];
  for (int i = threadIdx.x; i < 16 * 32; i += 64) lds[i] = (short)(100 * (i / 32) + (i % 32));
  __syncthreads();
  const int l = threadIdx.x, G = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const short* a = lds + (4 * G + q) * 32 + 4 * p;
  v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
  short* d;
  (void)hipMalloc(&d, 64 * 4 * 2);
  probe<<<1, 64>>>(d);
  short h[256];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) printf("lane %2d: %4d %4d %4d %4d\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
  return 0;
}
