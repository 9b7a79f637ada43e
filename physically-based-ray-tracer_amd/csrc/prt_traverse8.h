// prt_traverse8.h -- 8-wide compressed-BVH traversal (one lane = one ray), the default BLAS layout.
//
// Same contract as prt_traverse.h (hit rule, conservative boxes); the node format is Node8
// (bvh_build.h).  Per visited node: 5 x 16-B loads, 8 quantised child slabs, leaf children's
// triangles tested on the spot, interior hits kept as one (child_base, ordered 8-bit mask) group.
// The current group lives in registers; a group is pushed to the LDS stack only when a new node
// has interior hits while the current group still has unvisited children, so the stack never holds
// more than one entry per tree level.
#pragma once
#include "prt_traverse.h"

namespace prt {

// ray-invariant slab set-up for one node
struct Slab8 {
  float ax, ay, az;  // (p - O) * rD
  float bx, by, bz;  // 2^(e-127) * rD  (exact: power-of-two scale)
};

__device__ __forceinline__ float byte_f(uint32_t w, int k) { return (float)((w >> (8 * k)) & 0xFFu); }

// hit mask (physical slots) of the 8 children; near/far plane choice by the sign of rD
__device__ __forceinline__ uint32_t node8_hits(const uint4& a, const uint4& c, const uint4& d, const uint4& e,
                                               const V3& O, const V3& rD, float tlimit) {
  const float sx = __uint_as_float((a.w & 0xFFu) << 23), sy = __uint_as_float(((a.w >> 8) & 0xFFu) << 23),
              sz = __uint_as_float(((a.w >> 16) & 0xFFu) << 23);
  const float ax = (__uint_as_float(a.x) - O.x) * rD.x, ay = (__uint_as_float(a.y) - O.y) * rD.y,
              az = (__uint_as_float(a.z) - O.z) * rD.z;
  const float bx = sx * rD.x, by = sy * rD.y, bz = sz * rD.z;
  // near / far quantised planes per axis: words (lo0-3, lo4-7) / (hi0-3, hi4-7)
  const bool px = rD.x >= 0.0f, py = rD.y >= 0.0f, pz = rD.z >= 0.0f;
  const uint32_t nx0 = px ? c.x : d.z, nx1 = px ? c.y : d.w, fx0 = px ? d.z : c.x, fx1 = px ? d.w : c.y;
  const uint32_t ny0 = py ? c.z : e.x, ny1 = py ? c.w : e.y, fy0 = py ? e.x : c.z, fy1 = py ? e.y : c.w;
  const uint32_t nz0 = pz ? d.x : e.z, nz1 = pz ? d.y : e.w, fz0 = pz ? e.z : d.x, fz1 = pz ? e.w : d.y;
  uint32_t hits = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int b = k & 3;
    const uint32_t wnx = k < 4 ? nx0 : nx1, wny = k < 4 ? ny0 : ny1, wnz = k < 4 ? nz0 : nz1;
    const uint32_t wfx = k < 4 ? fx0 : fx1, wfy = k < 4 ? fy0 : fy1, wfz = k < 4 ? fz0 : fz1;
    const float tnx = __builtin_fmaf(byte_f(wnx, b), bx, ax), tfx = __builtin_fmaf(byte_f(wfx, b), bx, ax);
    const float tny = __builtin_fmaf(byte_f(wny, b), by, ay), tfy = __builtin_fmaf(byte_f(wfy, b), by, ay);
    const float tnz = __builtin_fmaf(byte_f(wnz, b), bz, az), tfz = __builtin_fmaf(byte_f(wfz, b), bz, az);
    const float tn = fmaxf(fmaxf(tnx, tny), fmaxf(tnz, 0.0f)) * kPadRatio;  // both pads (prt_traverse.h)
    const float tf = fminf(fminf(tfx, tfy), tfz);
    if (tn <= tf && tn <= tlimit) hits |= 1u << k;
  }
  return hits;
}

// physical-slot mask -> traversal-order mask (bit k ^ oct)
__device__ __forceinline__ uint32_t order_mask(uint32_t m, uint32_t oct) {
  if (oct & 1u) m = ((m & 0x55u) << 1) | ((m >> 1) & 0x55u);
  if (oct & 2u) m = ((m & 0x33u) << 2) | ((m >> 2) & 0x33u);
  if (oct & 4u) m = ((m & 0x0Fu) << 4) | ((m >> 4) & 0x0Fu);
  return m;
}

// One lane's traversal stack: levels [0, STACK) in LDS (stk[2 * level * BLOCK], one column per lane), deeper
// levels in the lane's HBM spill column (S.spill, level-major so a wave's entries of one level are contiguous;
// S.spill_levels levels, 0 = no spill: the host sizes both from the BVH depth, prt_api.cpp stack_depth)
struct LaneStack {
  uint32_t* lds;
  uint2* spill;
  uint32_t* ovf;  // overflow counter (SceneDev::diag)
  uint32_t tid, stride;
  int cap;  // STACK + spill levels
};
// a group that finds no free stack level is counted, never silently lost (the host sizes the stacks from the
// BVH depth, so the count stays 0; prt_stats.stack_overflows reports it and the Python mirror raises on it)
__device__ __forceinline__ void stack_overflow(uint32_t* ovf) {
#ifndef PRT_NO_OVF_COUNT  // A/B only
  if (ovf) atomicAdd(ovf, 1u);
#endif
}
template <int STACK, int BLOCK>
__device__ __forceinline__ LaneStack lane_stack(const SceneDev& S, uint32_t* lds) {
  LaneStack L;
  L.lds = lds;
  L.spill = S.spill;
  L.ovf = S.diag;
  L.tid = blockIdx.x * blockDim.x + threadIdx.x;
  L.stride = gridDim.x * blockDim.x;
  L.cap = STACK + (S.spill ? S.spill_levels : 0);
  return L;
}
template <int STACK, int BLOCK>
__device__ __forceinline__ void stack_put(const LaneStack& L, int lvl, uint32_t a, uint32_t b) {
  if (lvl < STACK) {
    L.lds[(2 * lvl) * BLOCK] = a;
    L.lds[(2 * lvl + 1) * BLOCK] = b;
  } else {
    L.spill[(size_t)(lvl - STACK) * L.stride + L.tid] = make_uint2(a, b);
  }
}
template <int STACK, int BLOCK>
__device__ __forceinline__ void stack_get(const LaneStack& L, int lvl, uint32_t& a, uint32_t& b) {
  if (lvl < STACK) {
    a = L.lds[(2 * lvl) * BLOCK];
    b = L.lds[(2 * lvl + 1) * BLOCK];
  } else {
    const uint2 v = L.spill[(size_t)(lvl - STACK) * L.stride + L.tid];
    a = v.x;
    b = v.y;
  }
}

template <int STACK, int BLOCK, bool ANY>
__device__ __forceinline__ bool blas_traverse8(const Node8* __restrict__ nodes, const TriMT* __restrict__ tris,
                                               uint32_t root, const V3& O, const V3& D, const V3& rD, uint32_t inst,
                                               Hit& h, const LaneStack& stk, int lvl0 = 0) {
  const uint32_t oct = (rD.x < 0.0f ? 1u : 0u) | (rD.y < 0.0f ? 2u : 0u) | (rD.z < 0.0f ? 4u : 0u);
  uint32_t gbase = 0, gmask = 0, gimask = 0;  // current group: unvisited interior children (ordered bits)
  uint32_t node = root;
  int sp = 0;
  while (true) {
    {
      const uint4* np = blas_node(nodes, node);
      const uint4 a = np[0], b = np[1];
      const uint32_t imask = a.w >> 24;
      const uint32_t hits = node8_hits(a, np[2], np[3], np[4], O, rD, h.t);
      uint32_t lhit = hits & ~imask;
      while (lhit) {  // leaf children: test their triangles now
        const uint32_t k = __builtin_ctz(lhit);
        lhit &= lhit - 1u;
        const uint32_t meta = ((k < 4 ? b.z : b.w) >> (8 * (k & 3))) & 0xFFu;
        const uint32_t first = b.y + (meta >> 3), cnt = meta & 7u;
        for (uint32_t i = 0; i < cnt; i++) {
          float t, u, v;
          uint32_t prim;
          if (mt_test(tris + first + i, O, D, t, u, v, prim)) {
            if (ANY) {
              if (t < h.t) return true;  // tiny_bvh.h:6594 (h.t holds tmax)
            } else if (t < h.t || (t == h.t && (inst < h.inst || (inst == h.inst && prim > h.prim)))) {
              h.t = t; h.u = u; h.v = v; h.prim = prim; h.inst = inst;
            }
          }
        }
      }
      const uint32_t ihit = hits & imask;
      if (ihit) {
        if (gmask && lvl0 + sp < stk.cap) {
          stack_put<STACK, BLOCK>(stk, lvl0 + sp, gbase, gmask | (gimask << 8));
          sp++;
        } else if (gmask) {
          stack_overflow(stk.ovf);
        }
        gbase = b.x;
        gmask = order_mask(ihit, oct);
        gimask = imask;
      }
    }
    if (!gmask) {
      if (sp == 0) break;
      sp--;
      uint32_t m;
      stack_get<STACK, BLOCK>(stk, lvl0 + sp, gbase, m);
      gmask = m & 0xFFu;
      gimask = m >> 8;
    }
    const uint32_t bit = __builtin_ctz(gmask);
    gmask &= gmask - 1u;
    const uint32_t k = bit ^ oct;
    node = gbase + __builtin_popcount(gimask & ((1u << k) - 1u));
  }
  return false;
}

// instance BVH walk (S.tlas): TLAS groups on the stack below, each hit instance's BLAS walked at once on the
// stack space above them (tiny_bvh.h:2500-2565 / 2611-2673 with an 8-wide TLAS; bvh_build.h build_tlas8)
template <int STACK, int BLOCK, bool ANY>
__device__ __forceinline__ bool tlas_traverse8(const SceneDev& S, const Ray& r, Hit& h, const LaneStack& stk) {
  const uint32_t oct = (r.rD.x < 0.0f ? 1u : 0u) | (r.rD.y < 0.0f ? 2u : 0u) | (r.rD.z < 0.0f ? 4u : 0u);
  uint32_t gbase = 0, gmask = 0, gimask = 0;
  uint32_t node = 0;
  int sp = 0;
  while (true) {
    {
      const uint4* np = reinterpret_cast<const uint4*>(S.tlas8 + node);
      const uint4 a = np[0], b = np[1];
      const uint32_t imask = a.w >> 24;
      const uint32_t hits = node8_hits(a, np[2], np[3], np[4], r.O, r.rD, h.t);
      uint32_t lh = order_mask(hits & ~imask, oct);
      while (lh) {  // instances of this node, near to far
        const uint32_t k = __builtin_ctz(lh) ^ oct;
        lh &= lh - 1u;
        const uint32_t i = S.tlas_slot[b.y + k];
        const InstDev& I = S.inst[i];
        const V3 Oi = xform_point(r.O, I.inv), Di = xform_vector(r.D, I.inv);
        const V3 rDi = v3(safercp(Di.x), safercp(Di.y), safercp(Di.z));
        if (blas_traverse8<STACK, BLOCK, ANY>(S.nodes8, S.tris, S.mesh[I.mesh].root, Oi, Di, rDi, i, h, stk, sp) &&
            ANY)
          return true;
      }
      const uint32_t ihit = hits & imask;
      if (ihit) {
        if (gmask && sp < stk.cap) {
          stack_put<STACK, BLOCK>(stk, sp, gbase, gmask | (gimask << 8));
          sp++;
        } else if (gmask) {
          stack_overflow(stk.ovf);
        }
        gbase = b.x;
        gmask = order_mask(ihit, oct);
        gimask = imask;
      }
    }
    if (!gmask) {
      if (sp == 0) break;
      sp--;
      uint32_t m;
      stack_get<STACK, BLOCK>(stk, sp, gbase, m);
      gmask = m & 0xFFu;
      gimask = m >> 8;
    }
    const uint32_t bit = __builtin_ctz(gmask);
    gmask &= gmask - 1u;
    const uint32_t k = bit ^ oct;
    node = gbase + __builtin_popcount(gimask & ((1u << k) - 1u));
  }
  return false;
}

template <int STACK, int BLOCK>
__device__ __forceinline__ Hit scene_closest8(const SceneDev& S, const Ray& r, float tmax, const LaneStack& stk) {
  Hit h;
  h.t = tmax; h.u = 0.0f; h.v = 0.0f; h.prim = 0; h.inst = 0;
  if (S.tlas) {
    (void)tlas_traverse8<STACK, BLOCK, false>(S, r, h, stk);
    return h;
  }
  for (int i = 0; i < S.ninst; i++) {
    const InstDev& I = S.inst[i];
    if (slab1(I.bmin, I.bmax, r.O, r.rD, h.t) >= kFar) continue;
    const V3 Oi = xform_point(r.O, I.inv), Di = xform_vector(r.D, I.inv);
    const V3 rDi = v3(safercp(Di.x), safercp(Di.y), safercp(Di.z));
    blas_traverse8<STACK, BLOCK, false>(S.nodes8, S.tris, S.mesh[I.mesh].root, Oi, Di, rDi, (uint32_t)i, h, stk);
  }
  return h;
}

template <int STACK, int BLOCK>
__device__ __forceinline__ bool scene_anyhit8(const SceneDev& S, const Ray& r, float tmax, const LaneStack& stk) {
  if (S.tlas) {
    Hit h;
    h.t = tmax; h.u = 0.0f; h.v = 0.0f; h.prim = 0; h.inst = 0;
    return tlas_traverse8<STACK, BLOCK, true>(S, r, h, stk);
  }
  for (int i = 0; i < S.ninst; i++) {
    const InstDev& I = S.inst[i];
    if (slab1(I.bmin, I.bmax, r.O, r.rD, tmax) >= kFar) continue;
    const V3 Oi = xform_point(r.O, I.inv), Di = xform_vector(r.D, I.inv);
    const V3 rDi = v3(safercp(Di.x), safercp(Di.y), safercp(Di.z));
    Hit h;
    h.t = tmax;
    if (blas_traverse8<STACK, BLOCK, true>(S.nodes8, S.tris, S.mesh[I.mesh].root, Oi, Di, rDi, 0u, h, stk)) return true;
  }
  return false;
}

// stack words per lane of the one-ray-per-lane query kernels (16 two-word groups: one per tree level)
constexpr int kQueryStack = 16;
constexpr int kQueryWords = 2 * kQueryStack;

}  // namespace prt
