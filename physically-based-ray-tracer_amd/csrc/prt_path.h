// prt_path.h -- device pieces of Renderer::Trace used by the wavefront shading kernels.
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

// The shadow ray towards light `light` (0-3: point light i, kLightDir: the directional light, kLightSpot: the
// spot) from hit point I, as Core/Renderer.cpp:216-310 builds it; L gets the unit direction and dl the squared
// distance (point) or the distance (directional / spot) that the contribution uses.  The shading kernel and the
// traversal kernel both call this, so a queued shadow ray is only (I, light) and rebuilds bit for bit.
constexpr uint32_t kLightDir = 4, kLightSpot = 5, kLightArea = 6;
__device__ __forceinline__ void light_ray(const SceneDev& S, uint32_t light, V3 I, Ray& r, float& tmax, V3& L,
                                          float& dl) {
  if (light < 4) {                                                                          // :216-257
    const int i = (int)light;
    float Lx = S.ppos[3 * i] - I.x, Ly = S.ppos[3 * i + 1] - I.y, Lz = S.ppos[3 * i + 2] - I.z;
    const float dsq = (Lx * Lx + Ly * Ly) + Lz * Lz;
    const float dist = sqrtf(dsq);
    const float invD = 1.0f / dist;  // _mm_rcp_ps restated as an exact reciprocal
    Lx = Lx * invD; Ly = Ly * invD; Lz = Lz * invD;
    L = v3(Lx, Ly, Lz);
    dl = dsq;
    r = make_ray(I + L * kEpsilon, L);
    tmax = dsq - kEpsilon;                                                                  // tmax = squared distance (:257)
    return;
  }
  const float* lp = (light == kLightSpot) ? S.spos : S.dpos;                                // :270-326
  L = v3(lp[0], lp[1], lp[2]) - I;
  const float distance = length(L);
  L = L / distance;
  dl = distance;
  r = make_ray(I + L * kEpsilon, L);
  tmax = distance - kEpsilon;
}

// Picks the shadow rays of `kind` (emit(k, light) per ray, in order; the traversal kernel rebuilds each ray with
// light_ray) and returns the BRDF value the reference evaluates for this light class (0 when !LIGHTED).  nk gets
// the factors each ray's unoccluded contribution f_k is a product of: f_k = colour * factor, rebuilt by
// nee_contrib with the same multiplies in the same order, so one float4 per item stands for up to four stored
// contributions.  Draws whichLight for point lights: the reference draws it after tracing the four shadow rays
// (:267), which consume no random numbers, so drawing it first keeps the stream and lets only the chosen light
// direction stay live.
template <class Emit>
__device__ __forceinline__ V3 nee_lights(const SceneDev& S, uint32_t fl, int kind, V3 I, V3 V, V3 N, const Material& m,
                                         uint32_t& seed, float4& nk, Emit&& emit) {
  if (kind == 0) {                                                                          // :216-269
    const int wl = (int)(random_float(seed) * 10) % 4;                                     // :267
    V3 Lw = v3(0.0f, 0.0f, 0.0f);
    float kf[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      Ray r;
      float tmax, dsq;
      V3 L;
      light_ray(S, (uint32_t)i, I, r, tmax, L, dsq);
      const float invD = 1.0f / sqrtf(dsq);  // the same exact reciprocal light_ray scaled L by
      float cosa = (N.x * L.x + N.y * L.y) + N.z * L.z;
      cosa = (cosa > 0.0f) ? cosa : 0.0f;  // _mm_max_ps(cosa, 0)
      kf[i] = invD * cosa;                 // f_i = colour_i * kf[i]
      if (i == wl) Lw = L;
      emit(i, (uint32_t)i);
    }
    nk = make_float4(kf[0], kf[1], kf[2], kf[3]);
    if (!(fl & kLighted)) return v3(0.0f, 0.0f, 0.0f);
    return eval_combined_brdf(N, Lw, V, m);
  }
  const uint32_t light = (kind == 2) ? kLightSpot : kLightDir;                              // :270-326
  Ray r;
  float tmax, distance;
  V3 L;
  light_ray(S, light, I, r, tmax, L, distance);
  const float cosa = smax(0.0f, dot(N, L));
  if (kind == 2) {  // f_0 = (colour * (1 / d^2)) * cos inside the cone (factor > 0.9), else 0
    const float factor = dot(L, v3(S.srot[0], S.srot[1], S.srot[2]));
    nk = make_float4(cosa, 1 / (distance * distance), ((double)factor > 0.9) ? 1.0f : 0.0f, 0.0f);
  } else {          // f_0 = colour * cos
    nk = make_float4(cosa, 0.0f, 0.0f, 0.0f);
  }
  emit(0, light);
  return (fl & kLighted) ? eval_combined_brdf(N, L, V, m) : v3(0.0f, 0.0f, 0.0f);
}

// shadow ray k's unoccluded contribution from nee_lights' factors (Core/Renderer.cpp:257-263,283-288,309-316)
__device__ __forceinline__ V3 nee_contrib(const SceneDev& S, int kind, int k, float4 nk) {
  if (kind == 0) {
    const float f = k == 0 ? nk.x : (k == 1 ? nk.y : (k == 2 ? nk.z : nk.w));
    return v3(S.pcol[3 * k] * f, S.pcol[3 * k + 1] * f, S.pcol[3 * k + 2] * f);
  }
  if (kind == 2) return (nk.z != 0.0f) ? v3(S.scol[0], S.scol[1], S.scol[2]) * nk.y * nk.x : v3(0.0f, 0.0f, 0.0f);
  return v3(S.dcol[0], S.dcol[1], S.dcol[2]) * nk.x;
}

// result after NEE: emissive + throughput(=1) * (BRDF * contribution), the reference's float order.
// vis bit i = shadow ray i unoccluded.
__device__ __forceinline__ V3 nee_resolve(const SceneDev& S, int kind, uint32_t vis, V3 e, V3 brdf, float4 nk,
                                          uint32_t fl) {
  V3 c = v3(0.0f, 0.0f, 0.0f);
  if (kind == 0) {
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (vis & (1u << i)) c = c + nee_contrib(S, 0, i, nk);
    c = c / 0.3f;
  } else {
    if (vis & 1u) c = nee_contrib(S, kind, 0, nk);
    if (kind == 1) c = c / 0.5f;
    else if (kind == 2) c = c / 0.2f;
  }
  const V3 add = (fl & kLighted) ? brdf * c : v3(0.0f, 0.0f, 0.0f);
  return e + v3(1.0f, 1.0f, 1.0f) * add;
}

// lobe pick + BRDF sampling (Core/Renderer.cpp:376-404).  Returns false when the path ends here.
// bp_out (optional) receives the lobe probability; it is left alone on the perfect-mirror fast path.
__device__ __forceinline__ bool sample_bounce(const Material& m, V3 V, V3 N, uint32_t& seed, V3& dir, V3& thr,
                                             float* bp_out = nullptr) {
  int type = 1;
  thr = v3(1.0f, 1.0f, 1.0f);
  if (m.metal == 1.0f && m.rough == 0.0f) type = 2;                                         // :376
  else {
    const float bp = brdf_probability(m, V, N);                                             // :380
    if (bp_out) *bp_out = bp;
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


// ---- dielectrics (Core/Renderer.cpp:331-372, refract :522-550).  The reference gates this branch on a
// material flag its Scene never sets (Core/Scene.cpp:193-197 tests modelIndex == -1); here an instance
// flagged PRT_MAT_DIELECTRIC takes it, restated literally (the refract() helper receives eta = n1/n2 as the
// material index, so entering rays bend by 1.46 and a negative k returns a zero direction).
struct Dielectric {
  Ray refl, refr;   // reflection ray, refraction ray (direction 0 when refract() reports total reflection)
  float fresnel;    // weight of the reflected radiance; 1 - fresnel weighs the refracted one
  bool has_refr;    // k > 0 (:349-357): the refracted ray is traced
};
PRT_HD V3 refract_ref(V3 D, V3 N, float eta) {                                             // :522-550
  const float cosi = clampf(dot(D, N), -1.0f, 1.0f);
  float etai = 1.0f, etat = eta;
  if (cosi > 0.0f) { const float t = etai; etai = etat; etat = t; }
  const float etaRatio = etai / etat;
  const float cosTheta = fabsf(cosi);
  const float k = 1.0f - etaRatio * etaRatio * (1.0f - cosTheta * cosTheta);
  if (k < 0.0f) return v3(0.0f, 0.0f, 0.0f);
  return etaRatio * (D - N * cosTheta) - N * sqrtf(k);
}
__device__ __forceinline__ Dielectric dielectric_split(V3 I, V3 D, V3 N) {
  Dielectric o;
  const float n1 = 1.0f, n2 = 1.46f;                                                        // :336-337
  const float cosTheta = clampf(-dot(D, N), 0.0f, 1.0f);                                   // :340
  o.refl = make_ray(I + N * kEpsilon, reflect(D, N));                                       // :343-346
  const float eta = n1 / n2;                                                                // :349
  const float k = 1.0f - eta * eta * (1.0f - cosTheta * cosTheta);                          // :350
  o.has_refr = k > 0.0f;
  o.refr = make_ray(I - N * kEpsilon, refract_ref(D, N, eta));                              // :353-358
  const float R0 = ((n1 - n2) / (n1 + n2)) * ((n1 - n2) / (n1 + n2));                      // :362
  o.fresnel = R0 + (1.0f - R0) * cr_pow(1.0f - cosTheta, 5.0f);                            // :363
  if (k <= 0.0f) o.fresnel = 1.0f;                                                          // :366
  return o;
}
// albedo * (fresnel * reflected + (1 - fresnel) * refracted), albedo = float3(1) (:369)
PRT_HD V3 dielectric_combine(float fresnel, V3 reflected, V3 refracted) {
  return v3(1.0f, 1.0f, 1.0f) * (fresnel * reflected + (1.0f - fresnel) * refracted);
}

// ---- area light (extension beyond the reference: Core/AreaLight.cpp defines the light but Trace never
// samples it).  One emitting parallelogram p0 + a*eu + b*ev, a, b in [0,1], radiance Le on the side of
// n = normalize(cross(eu, ev)) (both sides when two-sided).  Every shaded hit of a lit render samples it
// once (next-event estimation, 2 extra draws) and BRDF-sampled rays that reach it first see Le; the two
// strategies are combined with the power heuristic.  Paths end at the light; it casts no shadow for the
// reference's lights.  Same arithmetic in oracle/prt_oracle.c.
struct AreaLight {
  V3 p0, eu, ev, n, le;
  float area;
  int two_sided;
};
__device__ __forceinline__ AreaLight area_light(const SceneDev& S) {
  AreaLight A;
  A.p0 = v3(S.al[0], S.al[1], S.al[2]);
  A.eu = v3(S.al[3], S.al[4], S.al[5]);
  A.ev = v3(S.al[6], S.al[7], S.al[8]);
  A.n = v3(S.al[9], S.al[10], S.al[11]);
  A.le = v3(S.al[12], S.al[13], S.al[14]);
  A.area = S.al[15];
  A.two_sided = S.area_two_sided;
  return A;
}
// ray vs parallelogram (Moller-Trumbore on the triangle p0, p0+eu, p0+ev with a, b each in [0, 1]):
// t in (0, tmax) -> true, with cos_l = the emitting-side cosine (<= 0 means the back of a one-sided light)
PRT_HD bool area_hit(const AreaLight& A, V3 O, V3 D, float tmax, float& t, float& cos_l) {
  const V3 h = cross(D, A.ev);
  const float det = dot(A.eu, h);
  if (fabsf(det) < 1e-12f) return false;
  const float f = 1.0f / det;
  const V3 s = O - A.p0;
  const float a = f * dot(s, h);
  if (a < 0.0f || a > 1.0f) return false;
  const V3 q = cross(s, A.eu);
  const float b = f * dot(D, q);
  if (b < 0.0f || b > 1.0f) return false;
  t = f * dot(A.ev, q);
  if (!(t > 0.0f && t < tmax)) return false;
  cos_l = -dot(A.n, D);
  if (A.two_sided) cos_l = fabsf(cos_l);
  return true;
}
PRT_HD float mis_power(float a, float b) {  // a^2 / (a^2 + b^2); an infinite b (delta strategy) gives 0
  const float a2 = a * a, b2 = b * b;
  return a2 / (a2 + b2);
}
// solid-angle density of the BRDF sampling at this vertex (Core/Renderer.cpp:376-399): lobe pick p_spec,
// cosine hemisphere (BRDF.cpp:62-82), GGX VNDF (BRDF.cpp:224-269, alpha = roughness^2)
PRT_HD float brdf_pdf(const Material& m, V3 N, V3 V, V3 L, float p_spec) {
  const V3 Nn = normalize(N);
  const float NdotL = dot(Nn, L);
  if (NdotL <= 0.0f) return 0.0f;
  const float pd = NdotL * (1.0f / kPi);
  const V3 H = normalize(L + V);
  const float NdotV = smin(smax(0.00001f, dot(Nn, V)), 1.0f);
  const float NdotH = saturate(dot(Nn, H));
  const float alpha = m.rough * m.rough;
  const float a2 = smax(0.00001f, alpha * alpha);
  const float b = ((a2 - 1.0f) * NdotH * NdotH + 1.0f);
  const float D = a2 / (kPi * b * b);
  const float G1 = 2.0f * NdotV / (NdotV + sqrtf(a2 + (1.0f - a2) * (NdotV * NdotV)));
  const float ps = D * G1 / (4.0f * NdotV);
  return p_spec * ps + (1.0f - p_spec) * pd;
}
// the BRDF lobe probability used above: 1 for the perfect-mirror fast path (:376), else getBrdfProbability
PRT_HD bool delta_lobe(const Material& m) { return m.metal == 1.0f && m.rough == 0.0f; }


// next-event estimation of the area light at a shaded hit: false when the sample faces away (no ray);
// else the shadow ray, its tmax and the unoccluded contribution BRDF * Le * w_light / p_light
__device__ __forceinline__ bool area_nee(const AreaLight& A, V3 I, V3 N, V3 V, const Material& m, float xi1, float xi2,
                                         Ray& sr, float& tmax, V3& f) {
  const V3 y = A.p0 + xi1 * A.eu + xi2 * A.ev;
  V3 L = y - I;
  const float dsq = dot(L, L);
  const float dist = sqrtf(dsq);
  L = L / dist;
  float cos_l = -dot(A.n, L);
  if (A.two_sided) cos_l = fabsf(cos_l);
  if (!(cos_l > 0.0f) || !(dot(N, L) > 0.0f)) return false;
  const float pl = dsq / (A.area * cos_l);
  const float pb = brdf_pdf(m, N, V, L, brdf_probability(m, V, N));
  const float w = mis_power(pl, pb);
  f = eval_combined_brdf(N, L, V, m) * (A.le * (w / pl));
  sr = make_ray(I + L * kEpsilon, L);
  tmax = dist - kEpsilon;
  return true;
}
// radiance a ray sees when it reaches the light first: Le weighted against light sampling at the vertex
// that sampled it (pdf_prev = its brdf_pdf; kFar for camera rays, delta lobes, dielectric rays, unlit)
__device__ __forceinline__ V3 area_seen(const AreaLight& A, float t, float cos_l, float pdf_prev) {
  if (!(cos_l > 0.0f)) return v3(0.0f, 0.0f, 0.0f);
  if (pdf_prev >= kFar) return A.le;
  const float pl = (t * t) / (A.area * cos_l);
  return A.le * mis_power(pdf_prev, pl);
}

// RGBF32_to_RGB8 (template/precomp.h:310-315, scalar path)
__device__ __forceinline__ uint32_t pack1(float x) {
  const float mm = smin(1.0f, x);
  return mm > 0.0f ? (uint32_t)(255.0f * mm) : 0u;
}

}  // namespace prt
