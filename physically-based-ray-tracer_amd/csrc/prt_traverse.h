// prt_traverse.h -- single-ray TLAS -> BLAS traversal on CDNA4 (one lane = one ray).
//
// Replaces BVH::IntersectTLAS / IsOccludedTLAS (Core/tiny_bvh.h:2500-2565, 2611-2673) and the
// AVX2 BVH8_CPU::Intersect / IsOccluded (:6302-6474, :6477-6601).
//
// Hit rule (identical in the oracle): Moeller-Trumbore exactly as the BVH8_CPU leaf lane math
// (:6412-6440; det eps 1e-6, u in [0,1], v >= 0, u+v <= 1, t > 0; any-hit adds t < tmax), closest
// t wins; an equal t goes to the smaller instance, then to the LARGER prim -- what BVH8_CPU's leaf does with
// the two triangles of a quad sharing an edge (:6436 __bfind keeps the highest lane among equal minima, and
// the leaves hold primitives in ascending order).  Box tests are conservative (inflated boxes, padded slab
// interval), so the result does not depend on the BVH's shape.
//
// Shared pieces of the traversal kernels: ray / hit records, the leaf test, the instance-box slab.
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
// both pads on the near side: tn * kPadRatio <= tf accepts whatever tn * kNearPad <= tf * kFarPad accepts
// (kPadRatio < kNearPad / kFarPad), and tn * kPadRatio <= tlimit whatever tn * kNearPad <= tlimit does
constexpr float kPadRatio = 0.99998f;

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

__device__ __forceinline__ float slab1(const float* bmin, const float* bmax, const V3& O, const V3& rD, float tlimit) {
  float tx1 = (bmin[0] - O.x) * rD.x, tx2 = (bmax[0] - O.x) * rD.x;
  float ty1 = (bmin[1] - O.y) * rD.y, ty2 = (bmax[1] - O.y) * rD.y;
  float tz1 = (bmin[2] - O.z) * rD.z, tz2 = (bmax[2] - O.z) * rD.z;
  float a = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fmaxf(fminf(tz1, tz2), 0.0f)) * kNearPad;
  float b = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2)) * kFarPad;
  return (a <= b && a <= tlimit) ? a : kFar;
}

}  // namespace prt
