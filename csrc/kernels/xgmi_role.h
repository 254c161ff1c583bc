// Direct-xGMI collective "roles" (csrc/kernels/xgmi.hip): the device side of one phase collective
// over hipIpc-shared regions, written so that it runs either as its own launch or as the first
// `nblk` blocks of a compute kernel's launch (co-launch). A co-launched collective costs no launch,
// no stream fork/join and no cross-queue edge in the step's HIP graph: it moves its bytes over xGMI
// on CUs the compute blocks of the same launch leave idle.
//
// Region layout (identical on every rank, base = hipMalloc'd, exported by IPC):
//   [0, 4 KB) control: flags u32[kPhases][kMaxRanks] (flags[ph][src] written by rank src), epoch
//   u32[kPhases] (local), ticket u32[kPhases] (local), err u32 (bit r: timed out waiting for rank
//   r; bit 31: poisoned). [4 KB, ...) data.
//
// Phase protocol, per launch of phase ph with epoch e = epoch[ph] + 1:
//   enter: the first kSignalBlocks role blocks store e into flags[ph][rank] of every peer
//          (system-scope stores over xGMI), each after a SYSTEM-scope release fence; every role
//          block polls its own flags[ph][*] until each peer reached e (relaxed system-scope loads +
//          s_sleep; bounded by tmo wall-clock ticks: on timeout set err and its host-coherent mirror,
//          which the health monitor watches, and continue poisoned: gathers write NaN, a fused
//          Adam leaves the parameters at their last good values).
//          Memory-model argument: the published data of ph was written by launches that completed
//          before this one on the same stream. Each such launch ends with the dispatch packet's
//          release fence (agent scope in a captured graph), which writes every XCD's L2 back to the
//          memory side (the only point where the non-coherent per-XCD L2s meet), and the signal's
//          own system-scope release orders it after that at the scope the peers read at. Peers
//          read with system-scope loads (sc0 sc1, below), which miss in their own caches and are
//          served by this GPU's memory side. The argument is also checked end to end at start-up:
//          select_data_plane() compares graph-replayed steps on this plane against RCCL from one
//          snapshot and drops the plane on any mismatch (MIHVD_XGMI_DEBUG_STALE=1 injects stale
//          reads to show that the check fires).
//   move:  peer bytes are read with system-scope loads (buffer loads, sc0 sc1), which miss in this
//          GPU's caches for peer memory, so no line cached in an earlier epoch is returned.
//   exit:  the last role block to finish (device-scope ticket) publishes epoch[ph] = e.
// A rank enters phase ph only after every earlier launch on its stream completed, so "every peer
// entered ph at e" also means every peer finished reading what it read in earlier launches: the
// caller rewrites a published buffer only after a later phase (docs/ARCHITECTURE.md, "xGMI").
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace mihvd {

constexpr int kXgMaxRanks = 8;
constexpr int kXgPhases = 64;
constexpr int64_t kXgCtlBytes = 4096;
constexpr int64_t kXgFlagsOff = 0;                                  // u32[kPhases][kMaxRanks]
constexpr int64_t kXgEpochOff = kXgFlagsOff + kXgPhases * kXgMaxRanks * 4;
constexpr int64_t kXgTicketOff = kXgEpochOff + kXgPhases * 4;
constexpr int64_t kXgErrOff = kXgTicketOff + kXgPhases * 4;
constexpr unsigned kXgPoison = 0x80000000u;
constexpr int kXgAuxSys = 17;                  // sc0 | sc1: system-scope load
constexpr unsigned kXgSignalBlocks = 4;         // role blocks that signal (redundantly)
constexpr uint32_t kXgOob = 0xFFFFFFF0u;        // buffer offset past every range: load returns 0

enum CollKind : int { COLL_NONE = 0, COLL_GATHER = 1, COLL_REDUCE = 2 };

struct PeerTab {
  char* base[kXgMaxRanks];  // every rank's region; [rank] is this rank's own
};

// One prepared collective (kernel argument, passed by value; built on the host by xgmi.hip).
struct CollRole {
  PeerTab pt;
  int kind = COLL_NONE;
  int nblk = 0;             // role blocks: the first nblk linear block ids of the launch
  int ph = 0, rank = 0, world = 1;
  uint64_t tmo = 0;         // timeout in wall_clock64 ticks (100 MHz)
  // gather: rows [p*R, p*R + R) (capped at total_rows) of every peer p, byte columns
  // [col_off, col_off + col_bytes) of rows of `stride` bytes, buffer at region byte `off`
  int64_t off = 0, stride = 0, col_off = 0, col_bytes = 0;
  int R = 0, total_rows = 0;
  // reduce: out[i] = scale * sum_p peer_p[off + parity * slot_bytes + 4i] (rank order), n floats;
  // adam: the Adam update of the parameters of those gradients (aa), fused
  int64_t slot_bytes = 0, n = 0;
  float* out = nullptr;
  float scale = 1.f;
  int adam = 0;
  int bump = 1;             // with adam: block 0 advances the forward step counter (adam_step's bump)
  AdamArgs aa{};            // aa.shadow null: fp32 parameters only (the fp32 step has no bf16 copy)
  int dbg_stale = 0;        // debug (MIHVD_XGMI_DEBUG_STALE): gathers skip odd rows -> stale data
  unsigned* herr = nullptr; // host-coherent mirror of err (the health monitor's watched word)
};

// Host: the prepared role of descriptor id (xgmi.hip); id < 0 -> no role (nblk = 0).
CollRole xgmi_role_lookup(int64_t id);

}  // namespace mihvd

// The role code runs inside the MFMA kernels' launches and its fused Adam writes their operand
// format's shadow (common.h), so it is compiled in the kernels' namespace.
MIHVD_OPNS_BEGIN

__device__ __forceinline__ unsigned* xg_u32(char* base, int64_t off) { return (unsigned*)(base + off); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xg_rsrc(const char* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

typedef unsigned xg_u32x4 __attribute__((ext_vector_type(4)));

// Enter the phase (see the header). Returns the epoch; ok = false: poison the outputs.
__device__ __forceinline__ unsigned xg_enter(const CollRole& c, int bid, bool& ok) {
  __shared__ unsigned s_e, s_err;
  char* mine = c.pt.base[c.rank];
  const int t = threadIdx.x;
  if (t == 0) {
    const unsigned e =
        __hip_atomic_load(xg_u32(mine, kXgEpochOff) + c.ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    s_e = e;
    s_err = __hip_atomic_load(xg_u32(mine, kXgErrOff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((unsigned)bid < kXgSignalBlocks) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: before the peers can see e
      for (int p = 0; p < c.world; ++p)
        if (p != c.rank)
          __hip_atomic_store(xg_u32(c.pt.base[p], kXgFlagsOff) + c.ph * kXgMaxRanks + c.rank, e, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  const unsigned e = s_e;
  int good = s_err == 0u;
  if (good && t < c.world && t != c.rank) {
    const unsigned* f = xg_u32(mine, kXgFlagsOff) + c.ph * kXgMaxRanks + t;
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > c.tmo) {
        __hip_atomic_fetch_or(xg_u32(mine, kXgErrOff), (1u << t) | kXgPoison, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
        // the host's health monitor polls this copy (no PCIe atomic: any nonzero value is the signal)
        if (c.herr != nullptr)
          __hip_atomic_store(c.herr, (1u << t) | kXgPoison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        good = 0;
        break;
      }
    }
  }
  ok = __syncthreads_and(good) != 0;
  return e;
}

__device__ __forceinline__ void xg_exit(const CollRole& c, unsigned e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    char* mine = c.pt.base[c.rank];
    const unsigned tk =
        __hip_atomic_fetch_add(xg_u32(mine, kXgTicketOff) + c.ph, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tk == (unsigned)c.nblk - 1u) {
      __hip_atomic_store(xg_u32(mine, kXgTicketOff) + c.ph, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(xg_u32(mine, kXgEpochOff) + c.ph, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Gather: every unit (16 B) of every peer in flight at once per lane; this rank's own unit and
// absent ranks get an out-of-range offset (the load returns 0 without a memory access), so there
// is no branch around any load (a branch makes hipcc wait for each load before the next).
__device__ __forceinline__ void xg_gather(const CollRole& c, int bid, bool ok) {
  if (c.world == 1) return;  // a world of one: no peer rows (the phase entry/exit alone)
  const int64_t cu = c.col_bytes >> 4;
  const int64_t U = (int64_t)c.R * cu;
  const uint32_t span = (uint32_t)((int64_t)c.total_rows * c.stride);
  char* mine = c.pt.base[c.rank] + c.off;
  const int64_t nthreads = (int64_t)c.nblk * blockDim.x;
  for (int64_t i = (int64_t)bid * blockDim.x + threadIdx.x; i < U; i += nthreads) {
    const int64_t r = i / cu, cc = i - r * cu;
    xg_u32x4 v[kXgMaxRanks];
#pragma unroll
    for (int p = 0; p < kXgMaxRanks; ++p) {
      const bool live = p < c.world && p != c.rank;
      const uint32_t o = (uint32_t)(((int64_t)p * c.R + r) * c.stride + c.col_off + cc * 16);
      const char* b = c.pt.base[live ? p : c.rank] + c.off;
      v[p] = __builtin_amdgcn_raw_buffer_load_b128(xg_rsrc(b, span), live ? o : kXgOob, 0, kXgAuxSys);
    }
#pragma unroll
    for (int p = 0; p < kXgMaxRanks; ++p) {
      if (p >= c.world || p == c.rank) continue;
      const int64_t row = (int64_t)p * c.R + r;
      if (row >= c.total_rows || (c.dbg_stale && (r & 1))) continue;
      xg_u32x4 x = v[p];
      if (!ok) x = xg_u32x4{0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u};  // bf16 / f32 NaN
      *(xg_u32x4*)(mine + row * c.stride + c.col_off + cc * 16) = x;
    }
  }
}

// Reduce (+ Adam): sums in rank order; with adam the update of this rank's copy of the parameters
// (common.h adam4, the same code as adam_step) runs on the sum in registers; bid 0 advances the
// forward step counter (adam_step's bump). n is a multiple of 4 when adam is set.
__device__ __forceinline__ void xg_reduce(const CollRole& c, int bid, bool ok, unsigned e) {
  const int64_t off = c.off + (int64_t)(e & 1u) * c.slot_bytes;
  const uint32_t span = (uint32_t)(c.n * 4);
  const float nan = __uint_as_float(0x7FC00000u);
  AdamCoef ac{};
  if (c.adam) {
    ac = adam_coef((float)c.aa.state[ST_OPT], c.aa.lr, c.aa.b1, c.aa.b2, c.aa.eps, c.aa.gscale, c.aa.rule);
    if (c.bump && bid == 0 && threadIdx.x == 0) const_cast<int64_t*>(c.aa.state)[ST_FWD] += 1;
  }
  const int64_t n4 = c.n >> 2;
  const int64_t nthreads = (int64_t)c.nblk * blockDim.x;
  // p, m, v are loaded with the peers' gradients (one memory round trip per unit, not two: behind
  // the `adam && ok` branch they were issued only once the sum was formed); without Adam their
  // resources have no records and the loads return 0 without a memory access
  const uint32_t pspan = c.adam ? span : 0u;
  for (int64_t i = (int64_t)bid * blockDim.x + threadIdx.x; i < n4; i += nthreads) {
    xg_u32x4 v[kXgMaxRanks];
#pragma unroll
    for (int p = 0; p < kXgMaxRanks; ++p) {
      const bool live = p < c.world;
      v[p] = __builtin_amdgcn_raw_buffer_load_b128(xg_rsrc(c.pt.base[live ? p : c.rank] + off, span),
                                                   live ? (uint32_t)(i * 16) : kXgOob, 0, kXgAuxSys);
    }
    const xg_u32x4 pq = __builtin_amdgcn_raw_buffer_load_b128(xg_rsrc((const char*)c.aa.p, pspan), (uint32_t)(i * 16), 0, 0);
    const xg_u32x4 mq = __builtin_amdgcn_raw_buffer_load_b128(xg_rsrc((const char*)c.aa.m, pspan), (uint32_t)(i * 16), 0, 0);
    const xg_u32x4 vq = __builtin_amdgcn_raw_buffer_load_b128(xg_rsrc((const char*)c.aa.v, pspan), (uint32_t)(i * 16), 0, 0);
    float4 a = make_float4(__uint_as_float(v[0].x), __uint_as_float(v[0].y), __uint_as_float(v[0].z),
                           __uint_as_float(v[0].w));
#pragma unroll
    for (int p = 1; p < kXgMaxRanks; ++p) {
      if (p >= c.world) break;
      a.x += __uint_as_float(v[p].x);
      a.y += __uint_as_float(v[p].y);
      a.z += __uint_as_float(v[p].z);
      a.w += __uint_as_float(v[p].w);
    }
    a.x *= c.scale; a.y *= c.scale; a.z *= c.scale; a.w *= c.scale;
    if (!ok) a = make_float4(nan, nan, nan, nan);
    if (c.out) ((float4*)c.out)[i] = a;
    if (c.adam && ok) {  // poisoned: the parameters keep their last good values (no NaN update)
      float4 pp = make_float4(__uint_as_float(pq.x), __uint_as_float(pq.y), __uint_as_float(pq.z), __uint_as_float(pq.w));
      float4 mm = make_float4(__uint_as_float(mq.x), __uint_as_float(mq.y), __uint_as_float(mq.z), __uint_as_float(mq.w));
      float4 vv = make_float4(__uint_as_float(vq.x), __uint_as_float(vq.y), __uint_as_float(vq.z), __uint_as_float(vq.w));
      const uint2 sh = adam4(pp, mm, vv, a, ac);
      ((float4*)c.aa.p)[i] = pp;
      ((float4*)c.aa.m)[i] = mm;
      ((float4*)c.aa.v)[i] = vv;
      if (c.aa.shadow != nullptr) ((uint2*)c.aa.shadow)[i] = sh;
    }
  }
  for (int64_t i = (n4 << 2) + (int64_t)bid * blockDim.x + threadIdx.x; i < c.n; i += nthreads) {
    float a = 0.f;
    for (int p = 0; p < c.world; ++p)
      a += __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(xg_rsrc(c.pt.base[p] + off, span), (uint32_t)(i * 4), 0, kXgAuxSys));
    if (c.out) c.out[i] = ok ? a * c.scale : nan;
  }
}

// Split form (a dedicated launch pair instead of a co-launch): one block enters and leaves the phase
// (signal + wait for every peer + publish the epoch), and the data blocks of the NEXT launch on the
// same stream move the bytes without waiting. Only one block per rank polls, so several ranks
// sharing one GPU (the multi-rank tests) cannot starve a peer's kernels of wave slots with hundreds
// of spinning role blocks; stream order makes the data launch follow the completed entry.
__device__ __forceinline__ void coll_role_enter_exit(CollRole c) {
  c.nblk = 1;  // the ticket of this launch: one block
  bool ok;
  const unsigned e = xg_enter(c, 0, ok);
  xg_exit(c, e);
}

__device__ __forceinline__ void coll_role_data(const CollRole& c, int bid) {
  __shared__ unsigned s_e, s_err;
  if (threadIdx.x == 0) {
    char* mine = c.pt.base[c.rank];
    s_e = __hip_atomic_load(xg_u32(mine, kXgEpochOff) + c.ph, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_err = __hip_atomic_load(xg_u32(mine, kXgErrOff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const bool ok = s_err == 0u;
  if (c.kind == COLL_GATHER) xg_gather(c, bid, ok);
  else if (c.kind == COLL_REDUCE) xg_reduce(c, bid, ok, s_e);
}

// A gather role only (the host checked the kind): keeps the reduce + Adam code, and its registers,
// out of a host kernel that co-launches gathers alone (f32_conv1_fwd).
__device__ __forceinline__ void coll_gather_run(const CollRole& c, int bid) {
  bool ok;
  const unsigned e = xg_enter(c, bid, ok);
  xg_gather(c, bid, ok);
  xg_exit(c, e);
}

// Run the role as block `bid` of its nblk role blocks (any blockDim >= kXgMaxRanks threads).
__device__ __forceinline__ void coll_role_run(const CollRole& c, int bid) {
  bool ok;
  const unsigned e = xg_enter(c, bid, ok);
  if (c.kind == COLL_GATHER) xg_gather(c, bid, ok);
  else if (c.kind == COLL_REDUCE) xg_reduce(c, bid, ok, e);
  xg_exit(c, e);
}

MIHVD_OPNS_END
