// prt_queue.h -- work queues of the wavefront pipeline (prt_wave2.hip): sub-queue counters,
// consumer-side slot mapping, block-aggregated appends, XCD-partitioned dynamic fetch for the traversal kernels.
#pragma once
#include "prt_launch.h"

namespace prt {

enum : uint32_t { kStEndValue = 0, kStNeeEnd = 1, kStNeeCont = 2, kStMiss = 3 };
constexpr uint32_t kRiQueued = 1u << 24;  // rinfo: the shading kernel queued the item's next ray
constexpr uint32_t kRiEmissive = 1u << 25;  // rinfo: a hit's emissive term is nonzero (stored in ne; else +0)
constexpr uint32_t kRiFresh = 1u << 26;     // rinfo (merged pipeline): this slot was shaded in the last iteration

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t* qcounter(uint32_t* ctr, uint32_t iter, uint32_t which, uint32_t s) {
  return ctr + ((iter * 2u + which) * kNSub + s) * kCtrStride;
}

// LDS prefix table of the kNSub sub-queue counts; returns the total.  Call with uniform control flow.
__device__ __forceinline__ uint32_t load_prefix(const uint32_t* ctr, uint32_t iter, uint32_t which, uint32_t* pref) {
  if (threadIdx.x < 64) {
    const uint32_t l = threadIdx.x;
    uint32_t v = l < kNSub ? ctr[((iter * 2u + which) * kNSub + l) * kCtrStride] : 0u;
    for (int off = 1; off < 32; off <<= 1) {  // inclusive scan over the first 32 lanes
      const uint32_t o = __shfl_up(v, off, 64);
      if (l >= (uint32_t)off) v += o;
    }
    if (l < kNSub) pref[l + 1] = v;
    if (l == 0) pref[0] = 0;
  }
  __syncthreads();
  return pref[kNSub];
}
// global index g in [0, total) -> slot in the sub-queue layout (sub-queue s occupies [s*cap, s*cap+cnt_s))
__device__ __forceinline__ uint32_t map_slot(const uint32_t* pref, uint32_t g, uint32_t cap) {
  uint32_t lo = 0, hi = kNSub;
#pragma unroll
  for (int it = 0; it < 5; it++) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pref[mid] <= g) lo = mid; else hi = mid;
  }
  return lo * cap + (g - pref[lo]);
}

// Dynamic work fetch for the traversal kernels without a hot counter: the live range [0, total) is cut
// into kParts contiguous parts, each with its own fetch counter; a wave starts on the part of its XCD
// (HW_REG_XCC_ID) and steals from the others once that part is drained.  Returns false when all parts
// are drained.  Wave-uniform.
__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 7u;
}
__device__ __forceinline__ bool fetch_chunk(uint32_t* fctr, uint32_t total, uint32_t& part, uint32_t& base) {
  for (uint32_t tries = 0; tries < kParts; tries++) {
    const uint32_t lo = (uint32_t)(((uint64_t)total * part) / kParts);
    const uint32_t hi = (uint32_t)(((uint64_t)total * (part + 1)) / kParts);
    uint32_t off = 0;
    if (lane_id() == 0) off = (hi > lo) ? atomicAdd(fctr + part * kCtrStride, 64u) : 0xFFFFFFFFu;
    off = __shfl(off, 0, 64);
    if (off != 0xFFFFFFFFu && off < hi - lo) {
      base = lo + off;
      return true;
    }
    part = (part + 1) & (kParts - 1);
  }
  return false;
}
__device__ __forceinline__ uint32_t* fetch_counters(uint32_t* ctr, uint32_t iter, uint32_t which) {
  return ctr + ((size_t)(kMaxIters + 2) * 2 * kNSub + (iter * 2u + which) * kParts) * kCtrStride;
}

// block-aggregated append of n (0..4) entries per lane into one sub-queue; returns this lane's first
// index inside that sub-queue.  All threads of the block must call it.  sm: >= 8 words of LDS.
__device__ __forceinline__ uint32_t block_append(uint32_t* counter, uint32_t n, uint32_t* sm) {
  const uint64_t b1 = __ballot(n & 1u), b2 = __ballot((n >> 1) & 1u), b4 = __ballot((n >> 2) & 1u);
  const uint64_t lt = (1ull << lane_id()) - 1ull;
  const uint32_t before = (uint32_t)__popcll(b1 & lt) + 2u * (uint32_t)__popcll(b2 & lt) + 4u * (uint32_t)__popcll(b4 & lt);
  const uint32_t wtot = (uint32_t)__popcll(b1) + 2u * (uint32_t)__popcll(b2) + 4u * (uint32_t)__popcll(b4);
  const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane_id() == 0) sm[w] = wtot;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (uint32_t k = 0; k < nw; k++) tot += sm[k];
    sm[4] = tot ? atomicAdd(counter, tot) : 0u;
  }
  __syncthreads();
  uint32_t off = sm[4];
  for (uint32_t k = 0; k < w; k++) off += sm[k];
  __syncthreads();
  return off + before;
}

// hit record word: prim in the low S.pbits bits (enough for the largest mesh), instance above (prt_api.cpp
// checks that both fit in 32 bits)
__device__ __forceinline__ uint32_t pack_hit(const SceneDev& S, uint32_t prim, uint32_t inst) {
  return prim | (inst << S.pbits);
}
__device__ __forceinline__ uint32_t hit_prim(const SceneDev& S, uint32_t pk) { return pk & ((1u << S.pbits) - 1u); }
__device__ __forceinline__ uint32_t hit_inst(const SceneDev& S, uint32_t pk) { return pk >> S.pbits; }

// wave-uniform fetch of up to `want` consecutive live-range entries from the XCD-partitioned counters
__device__ __forceinline__ uint32_t fetch_some(uint32_t* fctr, uint32_t total, uint32_t& part, uint32_t* base,
                                               uint32_t want) {
  for (uint32_t tries = 0; tries < kParts; tries++) {
    const uint32_t lo = (uint32_t)(((uint64_t)total * part) / kParts);
    const uint32_t hi = (uint32_t)(((uint64_t)total * (part + 1)) / kParts);
    uint32_t off = 0xFFFFFFFFu;
    if (lane_id() == 0 && hi > lo) {
      // the wave's current part: straight to the atomic.  Other parts (stealing, end of launch): a plain
      // relaxed read first, so a drained part costs no atomic and the end of a launch does not queue
      // every wave's failing atomics on eight addresses
      uint32_t* ctr = fctr + part * kCtrStride;
      if (tries == 0 || __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hi - lo)
        off = atomicAdd(ctr, want);
    }
    off = __shfl(off, 0, 64);
    if (off != 0xFFFFFFFFu && off < hi - lo) {
      *base = lo + off;
      return min(want, hi - lo - off);
    }
    part = (part + 1) & (kParts - 1);
  }
  return 0;
}


}  // namespace prt
