// prt_traverse.h -- single-ray TLAS -> BLAS traversal on CDNA4 (one lane = one ray).
//
// Replaces BVH::IntersectTLAS / IsOccludedTLAS (Core/tiny_bvh.h:2500-2565, 2611-2673) and the
// AVX2 BVH8_CPU::Intersect / IsOccluded (:6302-6474, :6477-6601).
//
// Hit rule (identical in the oracle): Moeller-Trumbore exactly as the BVH8_CPU leaf lane math
// (:6412-6440; det eps 1e-6, u in [0,1], v >= 0, u+v <= 1, t > 0; any-hit adds t < tmax), closest
// t wins and equal t is broken by the smaller (instance, prim).  Box tests are conservative
// (inflated boxes, padded slab interval), so the result does not depend on the BVH's shape.
//
// Per-lane traversal stack lives in LDS as [depth][BLOCK] columns (bank-conflict-free: lane i
// always touches bank i mod 32).  Nodes are fetched as 7 x 16-B loads (bounds SoA + child refs).
#pragma once
#include "prt_math.h"
#include "prt_scene.h"

namespace prt {

struct Ray {
  V3 O, D, rD;
};
struct Hit {
  float t, u, v;
  uint32_t prim, inst;
};

// tinybvh::Ray ctor (Core/tiny_bvh.h:578-584): D normalised, rD = safercp(D)
__device__ __forceinline__ Ray make_ray(V3 origin, V3 dir) {
  Ray r;
  r.O = origin;
  r.D = normalize_bvh(dir);
  r.rD = v3(safercp(r.D.x), safercp(r.D.y), safercp(r.D.z));
  return r;
}

constexpr float kNearPad = 0.99999f;
constexpr float kFarPad = 1.00001f;

// BVH8_CPU leaf lane arithmetic, same operation order (Core/tiny_bvh.h:6413-6430)
__device__ __forceinline__ bool mt_test(const TriMT* __restrict__ tp, const V3& O, const V3& D, float& t_out,
                                        float& u_out, float& v_out, uint32_t& prim) {
  const float4* q = reinterpret_cast<const float4*>(tp);
  const float4 a = q[0], b = q[1], c = q[2];
  const float e1x = b.x, e1y = b.y, e1z = b.z, e2x = c.x, e2y = c.y, e2z = c.z;
  const float hx = D.y * e2z - D.z * e2y;
  const float hy = D.z * e2x - D.x * e2z;
  const float hz = D.x * e2y - D.y * e2x;
  const float sx = O.x - a.x, sy = O.y - a.y, sz = O.z - a.z;
  const float det = e1x * hx + e1y * hy + e1z * hz;
  const bool m1 = (det <= -0.000001f) || (det >= 0.000001f);
  const float inv_det = 1.0f / det;
  const float u = (sx * hx + sy * hy + sz * hz) * inv_det;
  const float qx = sy * e1z - sz * e1y;
  const float qy = sz * e1x - sx * e1z;
  const float qz = sx * e1y - sy * e1x;
  const float v = (D.x * qx + D.y * qy + D.z * qz) * inv_det;
  const float t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
  t_out = t;
  u_out = u;
  v_out = v;
  prim = __float_as_uint(a.w);
  return m1 && (u >= 0.0f) && (u <= 1.0f) && (v >= 0.0f) && (u + v <= 1.0f) && (t > 0.0f);
}

// conservative 4-wide slab test; returns near distances (kFar = miss)
__device__ __forceinline__ void slab4(const Node4* __restrict__ n, const V3& rD, const V3& orD, float tlimit,
                                      float tn[4], uint4& ch) {
  const float4* p = reinterpret_cast<const float4*>(n);
  const float4 lx = p[0], hx = p[1], ly = p[2], hy = p[3], lz = p[4], hz = p[5];
  ch = reinterpret_cast<const uint4*>(n)[6];
  const bool sx = rD.x >= 0.0f, sy = rD.y >= 0.0f, sz = rD.z >= 0.0f;
  const float4 nx = sx ? lx : hx, fx = sx ? hx : lx;
  const float4 ny = sy ? ly : hy, fy = sy ? hy : ly;
  const float4 nz = sz ? lz : hz, fz = sz ? hz : lz;
#define PRT_SLAB(c, i)                                                                                   \
  {                                                                                                      \
    float a = fmaxf(fmaxf(__builtin_fmaf(nx.c, rD.x, -orD.x), __builtin_fmaf(ny.c, rD.y, -orD.y)),     \
                    fmaxf(__builtin_fmaf(nz.c, rD.z, -orD.z), 0.0f));                                    \
    float b = fminf(fminf(__builtin_fmaf(fx.c, rD.x, -orD.x), __builtin_fmaf(fy.c, rD.y, -orD.y)),     \
                    __builtin_fmaf(fz.c, rD.z, -orD.z));                                                 \
    a = a * kNearPad;                                                                                    \
    tn[i] = (a <= b * kFarPad && a <= tlimit) ? a : kFar;                                                \
  }
  PRT_SLAB(x, 0)
  PRT_SLAB(y, 1)
  PRT_SLAB(z, 2)
  PRT_SLAB(w, 3)
#undef PRT_SLAB
}

__device__ __forceinline__ float slab1(const float* bmin, const float* bmax, const V3& O, const V3& rD, float tlimit) {
  float tx1 = (bmin[0] - O.x) * rD.x, tx2 = (bmax[0] - O.x) * rD.x;
  float ty1 = (bmin[1] - O.y) * rD.y, ty2 = (bmax[1] - O.y) * rD.y;
  float tz1 = (bmin[2] - O.z) * rD.z, tz2 = (bmax[2] - O.z) * rD.z;
  float a = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fmaxf(fminf(tz1, tz2), 0.0f)) * kNearPad;
  float b = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2)) * kFarPad;
  return (a <= b && a <= tlimit) ? a : kFar;
}

#define PRT_CSWAP(i, j)                         \
  if (d##j < d##i) {                            \
    float td = d##i; d##i = d##j; d##j = td;    \
    uint32_t tc = c##i; c##i = c##j; c##j = tc; \
  }

template <int STACK, int BLOCK>
__device__ __forceinline__ void blas_closest(const Node4* __restrict__ nodes, const TriMT* __restrict__ tris,
                                             uint32_t root, const V3& O, const V3& D, const V3& rD, uint32_t inst,
                                             Hit& h, uint32_t* __restrict__ stk) {
  const V3 orD = v3(O.x * rD.x, O.y * rD.y, O.z * rD.z);
  uint32_t node = root;
  int sp = 0;
  while (true) {
    if (!(node & kLeafBit)) {
      float tn[4];
      uint4 ch;
      slab4(nodes + node, rD, orD, h.t, tn, ch);
      float d0 = tn[0], d1 = tn[1], d2 = tn[2], d3 = tn[3];
      uint32_t c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
      PRT_CSWAP(0, 1) PRT_CSWAP(2, 3) PRT_CSWAP(0, 2) PRT_CSWAP(1, 3) PRT_CSWAP(1, 2)
      if (d3 < kFar && sp < STACK) { stk[sp * BLOCK] = c3; sp++; }
      if (d2 < kFar && sp < STACK) { stk[sp * BLOCK] = c2; sp++; }
      if (d1 < kFar && sp < STACK) { stk[sp * BLOCK] = c1; sp++; }
      if (d0 < kFar) { node = c0; continue; }
    } else {
      const uint32_t first = (node >> 2) & 0x1FFFFFFFu, cnt = (node & 3u) + 1u;
      for (uint32_t i = 0; i < cnt; i++) {
        float t, u, v;
        uint32_t prim;
        if (mt_test(tris + first + i, O, D, t, u, v, prim)) {
          if (t < h.t || (t == h.t && (inst < h.inst || (inst == h.inst && prim < h.prim)))) {
            h.t = t; h.u = u; h.v = v; h.prim = prim; h.inst = inst;
          }
        }
      }
    }
    if (sp == 0) break;
    sp--;
    node = stk[sp * BLOCK];
  }
}

template <int STACK, int BLOCK>
__device__ __forceinline__ bool blas_anyhit(const Node4* __restrict__ nodes, const TriMT* __restrict__ tris,
                                            uint32_t root, const V3& O, const V3& D, const V3& rD, float tmax,
                                            uint32_t* __restrict__ stk) {
  const V3 orD = v3(O.x * rD.x, O.y * rD.y, O.z * rD.z);
  uint32_t node = root;
  int sp = 0;
  while (true) {
    if (!(node & kLeafBit)) {
      float tn[4];
      uint4 ch;
      slab4(nodes + node, rD, orD, tmax, tn, ch);
      float d0 = tn[0], d1 = tn[1], d2 = tn[2], d3 = tn[3];
      uint32_t c0 = ch.x, c1 = ch.y, c2 = ch.z, c3 = ch.w;
      PRT_CSWAP(0, 1) PRT_CSWAP(2, 3) PRT_CSWAP(0, 2) PRT_CSWAP(1, 3) PRT_CSWAP(1, 2)
      if (d3 < kFar && sp < STACK) { stk[sp * BLOCK] = c3; sp++; }
      if (d2 < kFar && sp < STACK) { stk[sp * BLOCK] = c2; sp++; }
      if (d1 < kFar && sp < STACK) { stk[sp * BLOCK] = c1; sp++; }
      if (d0 < kFar) { node = c0; continue; }
    } else {
      const uint32_t first = (node >> 2) & 0x1FFFFFFFu, cnt = (node & 3u) + 1u;
      for (uint32_t i = 0; i < cnt; i++) {
        float t, u, v;
        uint32_t prim;
        if (mt_test(tris + first + i, O, D, t, u, v, prim) && t < tmax) return true;  // tiny_bvh.h:6594
      }
    }
    if (sp == 0) break;
    sp--;
    node = stk[sp * BLOCK];
  }
  return false;
}
#undef PRT_CSWAP

// BVH::IntersectTLAS: per instance, O and D through invTransform, D not renormalised (t stays world)
template <int STACK, int BLOCK>
__device__ __forceinline__ Hit scene_closest(const SceneDev& S, const Ray& r, float tmax, uint32_t* stk) {
  Hit h;
  h.t = tmax; h.u = 0.0f; h.v = 0.0f; h.prim = 0; h.inst = 0;
  for (int i = 0; i < S.ninst; i++) {
    const InstDev& I = S.inst[i];
    if (slab1(I.bmin, I.bmax, r.O, r.rD, h.t) >= kFar) continue;
    const V3 Oi = xform_point(r.O, I.inv), Di = xform_vector(r.D, I.inv);
    const V3 rDi = v3(safercp(Di.x), safercp(Di.y), safercp(Di.z));
    blas_closest<STACK, BLOCK>(S.nodes, S.tris, S.mesh[I.mesh].root, Oi, Di, rDi, (uint32_t)i, h, stk);
  }
  return h;
}

template <int STACK, int BLOCK>
__device__ __forceinline__ bool scene_anyhit(const SceneDev& S, const Ray& r, float tmax, uint32_t* stk) {
  for (int i = 0; i < S.ninst; i++) {
    const InstDev& I = S.inst[i];
    if (slab1(I.bmin, I.bmax, r.O, r.rD, tmax) >= kFar) continue;
    const V3 Oi = xform_point(r.O, I.inv), Di = xform_vector(r.D, I.inv);
    const V3 rDi = v3(safercp(Di.x), safercp(Di.y), safercp(Di.z));
    if (blas_anyhit<STACK, BLOCK>(S.nodes, S.tris, S.mesh[I.mesh].root, Oi, Di, rDi, tmax, stk)) return true;
  }
  return false;
}

}  // namespace prt
