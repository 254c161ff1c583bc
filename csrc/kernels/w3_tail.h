// dense/kernel Adam from dW3 tiles, as the tail of a compute launch (conv2_bwd, world size 1).
//
// At world size 1 nothing but the optimizer needs dW3 = a2^T dz ([3136][1024], K = batch). So the
// tail of the conv2_bwd launch multiplies the bf16 fc1 factors on MFMA tile by tile and applies
// Adam to W3 straight from the accumulators: against fc1_bwd storing dW3 and a plain Adam tail
// reading it back, 25.7 MB of the update's 96 MB of HBM traffic and fc1_bwd's 784 dW3 tiles go.
//
// Every wave is an independent worker (no LDS, no barriers): fc1_bwd's dgrad blocks leave the
// factors K-contiguous (a2T [3136][128], dzT [1024][128], zero past the batch), so each MFMA
// fragment is one 16-byte load straight from L2 (832 KB of factors, resident in every XCD's L2).
// A wave's tile is 32 (n) x 32 (j) of dW3^T: 4 K-steps x 4 fragment loads, 16 MFMAs, then Adam on
// 16 elements per lane from the accumulators. The next tile's factor loads are issued before this
// tile's Adam operands are waited for, and its operand loads right after this tile's stores, so
// each wave keeps up to 28 16-byte loads in flight; 8 such waves per CU cover the HBM latency.
// Waves of blocks with no conv work (on the CUs the conv roles leave idle) start at once and take
// the tiles [0, head) alone; then every wave of the launch shares [head, 3136) (static interleave).
//
// The MFMA accumulation order over K is fc1_wgrad's (ascending 32-wide steps; the zero rows past
// the batch add exact zeros) and every element runs adam4() of common.h, so this schedule is bitwise
// equal to fc1_wgrad + adam_step (tests/test_kernels_gpu.py).
#pragma once

#include "common.h"

MIHVD_OPNS_BEGIN

constexpr int W3T_N = 1024, W3T_K = 3136, W3T_KP = 128;  // factor rows are W3T_KP (= max batch) long
constexpr int W3T_TILES = (W3T_K / 32) * (W3T_N / 32);    // 3136 wave tiles of 32 x 32

struct W3TileTail {
  const u16* dzT;  // [1024][128] bf16: dz transposed, zero columns past the batch
  const u16* a2T;  // [3136][128] bf16: a2 transposed, likewise
  AdamArgs ad;     // p/m/v/shadow: the dense/kernel segments ([3136][1024]); state: ST_OPT
  float* gW3;      // nullptr, or also store dW3 there (tests)
  int first_free;  // blocks [first_free, grid) have no compute work ...
  int head;        // ... and alone take the tiles [0, head) first
};

struct W3Frags {
  uint4 a[4][2], b[4][2];  // [K step][16-row half]: dzT rows (n), a2T rows (j)
};
struct W3Ops {
  float4 p[2][2], m[2][2], v[2][2];  // [n half][j half]
};

// tile id -> (j0, n0): n fastest, so neighbouring tiles cover neighbouring columns of W3's rows
__device__ __forceinline__ void w3t_origin(int tile, int& j0, int& n0) {
  j0 = (tile >> 5) * 32;
  n0 = (tile & 31) * 32;
}

__device__ __forceinline__ void w3t_load_frags(const W3TileTail& wt, int tile, int lr, int lg, W3Frags& f) {
  int j0, n0;
  w3t_origin(tile, j0, n0);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f.a[ks][h] = *reinterpret_cast<const uint4*>(wt.dzT + (int64_t)(n0 + 16 * h + lr) * W3T_KP + 32 * ks + 8 * lg);
      f.b[ks][h] = *reinterpret_cast<const uint4*>(wt.a2T + (int64_t)(j0 + 16 * h + lr) * W3T_KP + 32 * ks + 8 * lg);
    }
}

// The optimizer stream (p, m, v, shadow: 84 MB) is read and written once per step: non-temporal
// accesses keep it from evicting the 1 MB of factors every wave re-reads from L2.
#ifndef MIHVD_W3T_NT
#define MIHVD_W3T_NT 1
#endif
__device__ __forceinline__ float4 w3t_ld(const float* p) {
#if MIHVD_W3T_NT
  typedef float f4v __attribute__((ext_vector_type(4)));
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return make_float4(v[0], v[1], v[2], v[3]);
#else
  return *reinterpret_cast<const float4*>(p);
#endif
}
__device__ __forceinline__ void w3t_st(float* p, const float4& x) {
#if MIHVD_W3T_NT
  typedef float f4v __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(f4v{x.x, x.y, x.z, x.w}, reinterpret_cast<f4v*>(p));
#else
  *reinterpret_cast<float4*>(p) = x;
#endif
}
__device__ __forceinline__ void w3t_st2(u16* p, const uint2& x) {
#if MIHVD_W3T_NT
  typedef unsigned int u2v __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store(u2v{x.x, x.y}, reinterpret_cast<u2v*>(p));
#else
  *reinterpret_cast<uint2*>(p) = x;
#endif
}

__device__ __forceinline__ int64_t w3t_off(int j0, int n0, int nh, int jh, int lr, int lg) {
  return (int64_t)(j0 + 16 * jh + lr) * W3T_N + n0 + 16 * nh + 4 * lg;
}

__device__ __forceinline__ void w3t_load_ops(const W3TileTail& wt, int tile, int lr, int lg, W3Ops& o) {
  int j0, n0;
  w3t_origin(tile, j0, n0);
#pragma unroll
  for (int nh = 0; nh < 2; ++nh)
#pragma unroll
    for (int jh = 0; jh < 2; ++jh) {
      const int64_t off = w3t_off(j0, n0, nh, jh, lr, lg);
      o.p[nh][jh] = w3t_ld(wt.ad.p + off);
      o.m[nh][jh] = w3t_ld(wt.ad.m + off);
      o.v[nh][jh] = w3t_ld(wt.ad.v + off);
    }
}

// This wave's tile sequence: the head range (blocks without conv work only), then the shared range.
struct W3TileSeq {
  int t, stride, end, shared_start, shared_stride;
  __device__ __forceinline__ void init(const W3TileTail& wt, int bx, int nblk, int wave, int nwb) {
    const int n_free = nblk - wt.first_free;
    const int head = n_free > 0 ? min(max(wt.head, 0), W3T_TILES) : 0;
    shared_start = head + bx * nwb + wave;
    shared_stride = nblk * nwb;
    if (bx >= wt.first_free && (bx - wt.first_free) * nwb + wave < head) {
      t = (bx - wt.first_free) * nwb + wave;
      stride = n_free * nwb;
      end = head;
    } else {
      t = shared_start;
      stride = shared_stride;
      end = W3T_TILES;
    }
  }
  __device__ __forceinline__ bool valid() const { return t < end; }
  __device__ __forceinline__ void advance() {
    t += stride;
    if (t >= end && end != W3T_TILES) {
      t = shared_start;
      stride = shared_stride;
      end = W3T_TILES;
    }
  }
};

// Every thread of the launch calls this after its compute role (if any); waves are independent.
__device__ __forceinline__ void w3_tail_run(const W3TileTail& wt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 15, lg = lane >> 4;
  W3TileSeq seq;
  seq.init(wt, (int)blockIdx.x, (int)gridDim.x, wave, (int)blockDim.x >> 6);
  if (!seq.valid()) return;
  const AdamCoef c = adam_coef((float)wt.ad.state[ST_OPT], wt.ad.lr, wt.ad.b1, wt.ad.b2, wt.ad.eps, wt.ad.gscale,
                               wt.ad.rule);
  W3Frags f;
  W3Ops o;
  w3t_load_frags(wt, seq.t, lr, lg, f);
  w3t_load_ops(wt, seq.t, lr, lg, o);
  while (true) {
    f32x4 acc[2][2];
#pragma unroll
    for (int nh = 0; nh < 2; ++nh) acc[nh][0] = acc[nh][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int nh = 0; nh < 2; ++nh)
#pragma unroll
        for (int jh = 0; jh < 2; ++jh)
          acc[nh][jh] = mfma16(__builtin_bit_cast(bf16x8, f.a[ks][nh]), __builtin_bit_cast(bf16x8, f.b[ks][jh]),
                               acc[nh][jh]);
    const int cur = seq.t;
    seq.advance();
    const bool more = seq.valid();
    if (more) w3t_load_frags(wt, seq.t, lr, lg, f);  // in flight during this tile's update
    int j0, n0;
    w3t_origin(cur, j0, n0);
#pragma unroll
    for (int nh = 0; nh < 2; ++nh)
#pragma unroll
      for (int jh = 0; jh < 2; ++jh) {
        const int64_t off = w3t_off(j0, n0, nh, jh, lr, lg);
        const float4 g = make_float4(acc[nh][jh][0], acc[nh][jh][1], acc[nh][jh][2], acc[nh][jh][3]);
        if (wt.gW3 != nullptr) *reinterpret_cast<float4*>(wt.gW3 + off) = g;
        const uint2 sh = adam4(o.p[nh][jh], o.m[nh][jh], o.v[nh][jh], g, c);
        w3t_st(wt.ad.p + off, o.p[nh][jh]);
        w3t_st(wt.ad.m + off, o.m[nh][jh]);
        w3t_st(wt.ad.v + off, o.v[nh][jh]);
        w3t_st2(wt.ad.shadow + off, sh);
      }
    if (!more) return;
    w3t_load_ops(wt, seq.t, lr, lg, o);
  }
}

MIHVD_OPNS_END
