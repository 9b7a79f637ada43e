// prt_path.h -- device pieces of Renderer::Trace shared by the megakernel and the wavefront pipeline.
#pragma once
#include "prt_kernels.h"
#include "prt_post.h"

namespace prt {

enum : uint32_t {
  kAA = 1u << 0, kAccumulate = 1u << 1, kGamma = 1u << 2, kNormalMap = 1u << 3,
  kSkybox = 1u << 4, kLighted = 1u << 5, kStochastic = 1u << 6
};
constexpr int kMaxBounces = 16;

// Camera::GetPrimaryRay (Core/Camera.cpp:113-139): screen plane, or the Panini projection when
// post-processing is on
__device__ __forceinline__ Ray primary_ray(const SceneDev& S, float x, float y, int W, int H) {
  const float u = x * (1.0f / (float)W);
  const float v = y * (1.0f / (float)H);
  const V3 camPos = v3(S.cam[0], S.cam[1], S.cam[2]);
  const V3 TL = v3(S.cam[3], S.cam[4], S.cam[5]), TR = v3(S.cam[6], S.cam[7], S.cam[8]),
           BL = v3(S.cam[9], S.cam[10], S.cam[11]);
  const V3 P = TL + u * (TR - TL) + v * (BL - TL);
  if (S.panini) {                                                                           // :125-134
    const V3 pd = panini_dir((2.0f * u) - 1.0f, 1.0f - (2.0f * v), S.pan_b, S.pan_d);
    const V3 c = pd * length(P - camPos);
    const V3 right = v3(S.basis[0], S.basis[1], S.basis[2]), up = v3(S.basis[3], S.basis[4], S.basis[5]),
             ahead = v3(S.basis[6], S.basis[7], S.basis[8]);
    return make_ray(camPos, normalize(right * c.x + up * c.y + ahead * c.z));
  }
  const V3 dir = normalize(P - camPos);
  return make_ray(camPos, dir);
}

// Renderer::Trace debug views (Core/Renderer.cpp:170-194)
__device__ __forceinline__ V3 debug_view(const SceneDev& S, int mode, const HitAttr& ha, uint32_t inst, uint32_t prim) {
  switch (mode) {
    case 1: return ha.m.base;
    case 4: return v3(ha.m.metal, ha.m.metal, ha.m.metal);
    case 5: return v3(ha.m.rough, ha.m.rough, ha.m.rough);
    case 6: return ha.m.emis;
    case 2: {
      const V3 g = geometry_normal(S, inst, prim);
      return v3(g.x + 1.0f, g.y + 1.0f, g.z + 1.0f) * 0.5f;
    }
    case 3: return v3(ha.N.x + 1.0f, ha.N.y + 1.0f, ha.N.z + 1.0f) * 0.5f;
    default: return v3(0.0f, 0.0f, 0.0f);
  }
}

// Next-event estimation set-up (Core/Renderer.cpp:198-326) split from its visibility tests.
// kind: 0 point (4 shadow rays), 1 directional, 2 spot, 3 non-stochastic directional.
__device__ __forceinline__ int nee_kind(uint32_t fl, uint32_t& seed) {
  if (!(fl & kStochastic)) return 3;
  const float pP = 0.3f, pD = 0.5f;
  const float xi = random_float(seed);                                                      // :210
  return (xi < pP) ? 0 : ((xi < pP + pD) ? 1 : 2);
}
__device__ __forceinline__ int nee_rays(int kind) { return kind == 0 ? 4 : 1; }

// Builds the shadow rays of `kind` (emit(k, ray, tmax, f_k) per ray, in order, with f_k the ray's
// unoccluded contribution before the pick-probability division) and returns the BRDF value the reference
// evaluates for this light class (0 when !LIGHTED).  Draws whichLight for point lights: the reference
// draws it after tracing the four shadow rays (:267), which consume no random numbers, so drawing it
// first keeps the stream and lets only the chosen light direction stay live.
template <class Emit>
__device__ __forceinline__ V3 nee_lights(const SceneDev& S, uint32_t fl, int kind, V3 I, V3 V, V3 N, const Material& m,
                                         uint32_t& seed, Emit&& emit) {
  if (kind == 0) {                                                                          // :216-269
    const int wl = (int)(random_float(seed) * 10) % 4;                                     // :267
    V3 Lw = v3(0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int i = 0; i < 4; i++) {
      float Lx = S.ppos[3 * i] - I.x, Ly = S.ppos[3 * i + 1] - I.y, Lz = S.ppos[3 * i + 2] - I.z;
      const float dsq = (Lx * Lx + Ly * Ly) + Lz * Lz;
      const float dist = sqrtf(dsq);
      const float invD = 1.0f / dist;  // _mm_rcp_ps restated as an exact reciprocal
      Lx = Lx * invD; Ly = Ly * invD; Lz = Lz * invD;
      float cosa = (N.x * Lx + N.y * Ly) + N.z * Lz;
      cosa = (cosa > 0.0f) ? cosa : 0.0f;  // _mm_max_ps(cosa, 0)
      const float k = invD * cosa;
      const V3 L = v3(Lx, Ly, Lz);
      if (i == wl) Lw = L;
      emit(i, make_ray(I + L * kEpsilon, L), dsq - kEpsilon,                                // tmax = squared distance (:257)
           v3(S.pcol[3 * i] * k, S.pcol[3 * i + 1] * k, S.pcol[3 * i + 2] * k));
    }
    if (!(fl & kLighted)) return v3(0.0f, 0.0f, 0.0f);
    return eval_combined_brdf(N, Lw, V, m);
  }
  const float* lp = (kind == 2) ? S.spos : S.dpos;                                          // :270-326
  const float* lc = (kind == 2) ? S.scol : S.dcol;
  V3 L = v3(lp[0], lp[1], lp[2]) - I;
  const float distance = length(L);
  L = L / distance;
  const float cosa = smax(0.0f, dot(N, L));
  V3 f0;
  if (kind == 2) {
    const float factor = dot(L, v3(S.srot[0], S.srot[1], S.srot[2]));
    f0 = ((double)factor > 0.9) ? v3(lc[0], lc[1], lc[2]) * (1 / (distance * distance)) * cosa
                                : v3(0.0f, 0.0f, 0.0f);
  } else {
    f0 = v3(lc[0], lc[1], lc[2]) * cosa;
  }
  emit(0, make_ray(I + L * kEpsilon, L), distance - kEpsilon, f0);
  return (fl & kLighted) ? eval_combined_brdf(N, L, V, m) : v3(0.0f, 0.0f, 0.0f);
}

// result after NEE: emissive + throughput(=1) * (BRDF * contribution), the reference's float order.
// vis bit i = shadow ray i unoccluded.
__device__ __forceinline__ V3 nee_resolve(int kind, uint32_t vis, V3 e, V3 brdf, const V3* f, uint32_t fl) {
  V3 c = v3(0.0f, 0.0f, 0.0f);
  if (kind == 0) {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (vis & (1u << i)) c = c + f[i];
    c = c / 0.3f;
  } else {
    if (vis & 1u) c = f[0];
    if (kind == 1) c = c / 0.5f;
    else if (kind == 2) c = c / 0.2f;
  }
  const V3 add = (fl & kLighted) ? brdf * c : v3(0.0f, 0.0f, 0.0f);
  return e + v3(1.0f, 1.0f, 1.0f) * add;
}

// lobe pick + BRDF sampling (Core/Renderer.cpp:376-404).  Returns false when the path ends here.
__device__ __forceinline__ bool sample_bounce(const Material& m, V3 V, V3 N, uint32_t& seed, V3& dir, V3& thr) {
  int type = 1;
  thr = v3(1.0f, 1.0f, 1.0f);
  if (m.metal == 1.0f && m.rough == 0.0f) type = 2;                                         // :376
  else {
    const float bp = brdf_probability(m, V, N);                                             // :380
    if (random_float(seed) < bp) { type = 2; thr = thr / bp; }
    else { type = 1; thr = thr / (1.0f - bp); }
  }
  V3 wgt = v3(1.0f, 1.0f, 1.0f);
  V2 u;
  u.x = random_float(seed);                                                                 // :396
  u.y = random_float(seed);
  if (!eval_indirect_brdf(u, N, V, m, type, dir, wgt)) return false;                       // :398
  thr = thr * wgt;
  return true;
}

// RGBF32_to_RGB8 (template/precomp.h:310-315, scalar path)
__device__ __forceinline__ uint32_t pack1(float x) {
  const float mm = smin(1.0f, x);
  return mm > 0.0f ? (uint32_t)(255.0f * mm) : 0u;
}

}  // namespace prt
