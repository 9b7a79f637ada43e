// prt_bounce.h -- one shading task of an item: the per-item body of the streaming engine (prt_stream.hip).
// (Fusing the merged pipeline's k_resolve2 / k_miss2 / k_shade2 into one launch around this body was
// measured slower, 2.91 vs 2.32 ms per C4 frame: one pass over the larger P(i-1) set at 3-4 waves/SIMD
// with spills, against three lean passes.)
//
// A task does, for one item, what Renderer::Trace does between two closest-hit queries
// (Core/Renderer.cpp:150-406): first the NEE resolve of the previous bounce (its shadow rays are
// traced), then the hit of the closest ray in flight -- sky or 0 on a miss (:159), the debug colour
// (:170-194), or the BRDF shading with the NEE set-up (shadow rays into the item's four slots
// sho/shd[4 item + k]) and the sampled bounce or, when path 1 ends with AA, path 2's primary ray.
// Every random number of the item is drawn here, in the reference order.
// LD supplies the loads of the per-item state (sc1 loads inside the streaming engine's launch; PlainLoads
// where a launch boundary separates producer and consumer).
#pragma once
#include "prt_launch.h"
#include "prt_path.h"
#include "prt_queue.h"

namespace prt {

constexpr uint32_t kHitPending = 1u << 9;  // info: a closest-hit ray of the item is in flight

// the sky lookup's double-precision atan2 / acos need ~70 VGPRs more than the rest of the task; as a real
// call they no longer set the register budget of every shading task (misses only)
__device__ __noinline__ V3 sky_call(const SceneDev& S, V3 D) { return sample_sky(S, D); }

struct PlainLoads {
  static __device__ __forceinline__ uint32_t u32(const uint32_t* p) { return *p; }
  static __device__ __forceinline__ float4 f4(const float4* a, uint32_t i) { return a[i]; }
};

// the path of `item` ends with value L at `depth` (k_resolve2's tail): result + L * throughput up the
// stack (:404), then path-1 radiance kept for AA (s1) or the frame value written.  R[depth-1] may be
// handed in from registers (top) when it was stored by this same task.  Returns true when the item is done.
template <class LD>
__device__ __forceinline__ bool end_path(const TraceArgs& A, const WaveBufs& B, uint32_t item, V3 L, uint32_t depth,
                                         uint32_t path, bool have_top, V3 top, float4& s1, float4* __restrict__ out) {
  for (int k = (int)depth - 1; k >= 0; k--) {
    const uint32_t e = (uint32_t)k * B.n + item;
    V3 Rk;
    if (have_top && k == (int)depth - 1) {
      Rk = top;
    } else {
      const float4 r = LD::f4(B.R, e);
      Rk = v3(r.x, r.y, r.z);
    }
    const float4 Tk = LD::f4(B.T, e);
    L = Rk + L * v3(Tk.x, Tk.y, Tk.z);
  }
  if (path == 0 && (A.flags & kAA)) {
    s1.x = L.x; s1.y = L.y; s1.z = L.z;
    return false;
  }
  V3 res = (A.flags & kAA) ? 0.5f * (v3(s1.x, s1.y, s1.z) + L) : L;                         // :65
  if (A.flags & kGamma) res = v3(sqrtf(res.x), sqrtf(res.y), sqrtf(res.z));                   // :73-79
  out[item] = make_float4(res.x, res.y, res.z, s1.w);
  return true;
}

// path 2's primary ray (its jitter was drawn at init, :61)
__device__ __forceinline__ void start_path2s(const SceneDev& S, const TraceArgs& A, const TileMap& M, const WaveBufs& B,
                                             uint32_t item) {
  const uint32_t r = item % M.items;
  int32_t x, y;
  item_pixel(M, r, x, y);
  const float2 j = B.jit[item];  // written by the init launch only
  const Ray r2 = primary_ray(S, (float)x + j.x, (float)y + j.y, A.W, A.H);
  B.ro[item] = make_float4(r2.O.x, r2.O.y, r2.O.z, 0.0f);
  B.rd[item] = make_float4(r2.D.x, r2.D.y, r2.D.z, 0.0f);
}

// one shading task: NEE resolve of the previous bounce (k_resolve2), then the pending hit (k_miss2 +
// k_shade2 / k_shade2_debug).  Out: done (frame value written), rays queued (hasC closest + nS shadow).
template <class LD>
__device__ __forceinline__ void shade_item(const SceneDev& S, const TraceArgs& A, const TileMap& M, const WaveBufs& B,
                                           uint32_t item, float4* __restrict__ out, bool first, bool& done,
                                           uint32_t& hasC, uint32_t& nS) {
  const uint32_t fl = A.flags;
  // per-item state is loaded where a branch needs it (loading all of it up front costs spills)
  const uint32_t info = first ? kHitPending : LD::u32(B.info + item);
  const uint32_t ri = first ? 0u : LD::u32(B.rinfo + item);
  float4 s1 = LD::f4(B.s1, item);
  bool s1dirty = false;
  bool have_top = false;
  V3 top = v3(0.0f, 0.0f, 0.0f);
  const uint32_t st = (ri >> 16) & 3u;
  if (st == kStNeeEnd || st == kStNeeCont) {
    const uint32_t depth = ri & 0xFFu, path = (ri >> 8) & 1u, kind = (ri >> 20) & 3u;
    const float4 ne = LD::f4(B.ne, item), nb = LD::f4(B.nb, item);
    const uint32_t vw = LD::u32(B.vis + item);
    const uint32_t vis = ((vw & 0xFFu) ? 1u : 0u) | ((vw & 0xFF00u) ? 2u : 0u) | ((vw & 0xFF0000u) ? 4u : 0u) |
                         ((vw & 0xFF000000u) ? 8u : 0u);
    V3 f[4];
    const uint32_t nr = kind == 0 ? 4u : 1u;
    for (uint32_t k = 0; k < 4; k++) {
      if (k < nr) {
        const float4 fk = LD::f4(B.nf, 4u * item + k);
        f[k] = v3(fk.x, fk.y, fk.z);
      } else {
        f[k] = v3(0.0f, 0.0f, 0.0f);
      }
    }
    const V3 result = nee_resolve((int)kind, vis, v3(ne.x, ne.y, ne.z), v3(nb.x, nb.y, nb.z), f, fl);
    if (st == kStNeeCont) {
      B.R[(size_t)depth * B.n + item] = make_float4(result.x, result.y, result.z, 0.0f);
      have_top = true;
      top = result;
    } else {
      done = end_path<LD>(A, B, item, result, depth, path, false, top, s1, out);
      s1dirty |= !done;  // path-1 radiance kept
    }
  }
  uint32_t ninfo = info & ~kHitPending, nri = 0;
  if (info & kHitPending) {
    const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u;
    const float4 hh = LD::f4(B.hit, item);
    if ((info & 0x1FFu) == 0) {  // r1.hit.t
      s1.w = hh.x;
      s1dirty = true;
    }
    bool ended = false;
    V3 L = v3(0.0f, 0.0f, 0.0f);
    if (hh.x >= kFar) {                                                                       // :159
      if (fl & kSkybox) {
        const float4 d = LD::f4(B.rd, item);
        L = sky_call(S, v3(d.x, d.y, d.z));
      }
      ended = true;
    } else if (A.mode != 0) {                                                                 // :170-194
      const uint32_t pk = __float_as_uint(hh.w);
      const HitAttr ha = hit_attributes(S, pk >> 26, pk & 0x03FFFFFFu, hh.y, hh.z, (fl & kNormalMap) != 0);
      L = debug_view(S, A.mode, ha, pk >> 26, pk & 0x03FFFFFFu);
      ended = true;
    } else {
      uint32_t seed = LD::u32(B.seed + item);
      const int kind = nee_kind(fl, seed);                                                    // :198-214
      const float4 o = LD::f4(B.ro, item), d = LD::f4(B.rd, item);
      const V3 D = v3(d.x, d.y, d.z);
      const uint32_t pk = __float_as_uint(hh.w);
      const V3 I = v3(o.x, o.y, o.z) + hh.x * D;                                               // tiny_bvh.h:586
      const V3 V = -D;
      const HitAttr ha = hit_attributes(S, pk >> 26, pk & 0x03FFFFFFu, hh.y, hh.z, (fl & kNormalMap) != 0);
      const V3 e = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * ha.m.emis;                  // :196
      B.ne[item] = make_float4(e.x, e.y, e.z, 0.0f);
      const V3 brdf = nee_lights(S, fl, kind, I, V, ha.N, ha.m, seed, [&](int k, const Ray& sr, float tmax, V3 fk) {
        const uint32_t sk = 4u * item + (uint32_t)k;
        B.sho[sk] = make_float4(sr.O.x, sr.O.y, sr.O.z, tmax);
        B.shd[sk] = make_float4(sr.D.x, sr.D.y, sr.D.z, 0.0f);
        B.nf[sk] = make_float4(fk.x, fk.y, fk.z, 0.0f);
      });
      nS = (uint32_t)nee_rays(kind);
      B.nb[item] = make_float4(brdf.x, brdf.y, brdf.z, 0.0f);
      B.vis[item] = 0u;
      uint32_t status = kStNeeEnd;
      if ((int)depth != A.bounces - 1) {                                                      // :329
        V3 dir, thr;
        if (sample_bounce(ha.m, V, ha.N, seed, dir, thr)) {                                   // :376-399
          status = kStNeeCont;
          B.T[(size_t)depth * B.n + item] = make_float4(thr.x, thr.y, thr.z, 0.0f);
          const Ray nr2 = make_ray(I + dir * kEpsilon, dir);                                  // :404
          B.ro[item] = make_float4(nr2.O.x, nr2.O.y, nr2.O.z, 0.0f);
          B.rd[item] = make_float4(nr2.D.x, nr2.D.y, nr2.D.z, 0.0f);
          ninfo = (depth + 1u) | (path << 8) | kHitPending;
          hasC = 1;
        }
      }
      B.seed[item] = seed;
      nri = depth | (path << 8) | (status << 16) | ((uint32_t)kind << 20);
      if (status == kStNeeEnd && path == 0 && (fl & kAA)) {  // path 2 starts beside path 1's last NEE
        start_path2s(S, A, M, B, item);
        ninfo = (1u << 8) | kHitPending;
        hasC = 1;
      }
    }
    if (ended) {
      done = end_path<LD>(A, B, item, L, depth, path, have_top && depth > 0, top, s1, out);
      if (!done) {  // path 1 of an AA pair: path 2 next
        s1dirty = true;
        start_path2s(S, A, M, B, item);
        ninfo = (1u << 8) | kHitPending;
        hasC = 1;
      }
    }
  }
  if (s1dirty) B.s1[item] = s1;
  B.info[item] = ninfo;
  B.rinfo[item] = nri;
}

}  // namespace prt
