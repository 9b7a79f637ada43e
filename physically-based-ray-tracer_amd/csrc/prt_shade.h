// prt_shade.h -- hit-attribute reconstruction, GGX/Lambert BRDF and sky, device side.
//
// Restates, with the reference's float expression order:
//   Scene::GetGeometryNormal / GetShadingNormal / GetMaterialBRDF  Core/Scene.cpp:47-218,225-263
//   BRDF::evalCombinedBRDF / evalIndirectCombinedBRDF / getBrdfProbability  Core/BRDF.cpp:16-526
//   Camera::SampleSkybox                                            Core/Camera.cpp:43-74
#pragma once
#include "prt_math.h"
#include "prt_scene.h"

namespace prt {

struct Material {  // MaterialProperties (Core/BRDF.h:165-176); transmissivness/opacity are never set
  V3 base;
  float metal;
  V3 emis;
  float rough;
};

struct BrdfData {  // BrdfData (Core/BRDF.h:178-208), fields the hot path reads
  V3 specF0, diffR;
  float alpha, alpha2;
  V3 F;
  float NdotL, NdotV, LdotH, NdotH, VdotH;
  bool Vback, Lback;
};

__device__ __forceinline__ float luminance(V3 c) { return dot(c, v3(0.2126f, 0.7152f, 0.0722f)); }  // :16-19
__device__ __forceinline__ V3 specular_f0(V3 base, float metal) {                                   // :21-30
  return lerp(v3(kMinDielectricsF0, kMinDielectricsF0, kMinDielectricsF0), base, metal);
}
__device__ __forceinline__ V3 diffuse_reflectance(V3 base, float metal) { return base * (1.0f - metal); }  // :32-35
__device__ __forceinline__ float shadowed_f90(V3 F0) {                                                      // :100-104
  const float t = (1.0f / kMinDielectricsF0);
  return smin(1.0f, t * luminance(F0));
}
__device__ __forceinline__ V3 fresnel_schlick(V3 f0, float f90, float NdotS) {  // :84-87
  const float p = pow5(1.0f - NdotS);
  return f0 + v3(f90 - f0.x, f90 - f0.y, f90 - f0.z) * p;
}
__device__ __forceinline__ float ggx_d(float a2, float NdotH) {  // :218-222
  float b = ((a2 - 1.0f) * NdotH * NdotH + 1.0f);
  return a2 / (kPi * b * b);
}
__device__ __forceinline__ float smith_g2_lagarde(float a2, float NdotL, float NdotV) {  // :170-175
  float a = NdotV * sqrtf(a2 + NdotL * (NdotL - a2 * NdotL));
  float b = NdotL * sqrtf(a2 + NdotV * (NdotV - a2 * NdotV));
  return 0.5f / (a + b);
}
__device__ __forceinline__ BrdfData prepare_brdf(V3 N, V3 L, V3 V, const Material& m) {  // :398-437
  BrdfData d;
  const V3 H = normalize(L + V);
  const float NdotL = dot(N, L), NdotV = dot(N, V);
  d.Vback = (NdotV <= 0.0f);
  d.Lback = (NdotL <= 0.0f);
  d.NdotL = smin(smax(0.00001f, NdotL), 1.0f);
  d.NdotV = smin(smax(0.00001f, NdotV), 1.0f);
  d.LdotH = saturate(dot(L, H));
  d.NdotH = saturate(dot(N, H));
  d.VdotH = saturate(dot(V, H));
  d.specF0 = specular_f0(m.base, m.metal);
  d.diffR = diffuse_reflectance(m.base, m.metal);
  d.alpha = m.rough * m.rough;
  d.alpha2 = d.alpha * d.alpha;
  d.F = fresnel_schlick(d.specF0, shadowed_f90(d.specF0), d.LdotH);
  return d;
}
// evalCombinedBRDF :439-452 = (1 - F) * Lambert + GGX microfacet (G2 pre-divided, :385-396)
__device__ __forceinline__ V3 eval_combined_brdf(V3 N, V3 L, V3 V, const Material& m) {
  const BrdfData d = prepare_brdf(N, L, V, m);
  if (d.Vback || d.Lback) return v3(0.0f, 0.0f, 0.0f);
  const float D = ggx_d(smax(0.00001f, d.alpha2), d.NdotH);
  const float G2 = smith_g2_lagarde(d.alpha2, d.NdotL, d.NdotV);
  const V3 spec = d.F * (G2 * D * d.NdotL);
  const V3 diff = d.diffR * ((1.0f / kPi) * d.NdotL);
  return one_minus(d.F) * diff + spec;
}
__device__ __forceinline__ Q4 rotation_to_z(V3 in) {  // :43-49
  Q4 r;
  if (in.z < -0.99999f) { r.x = 1.0f; r.y = 0.0f; r.z = 0.0f; r.w = 0.0f; return r; }
  const float qx = in.y, qy = -in.x, qz = 0.0f, qw = 1.0f + in.z;
  const float inv = 1.0f / sqrtf(qx * qx + qy * qy + qz * qz + qw * qw);
  r.x = qx * inv; r.y = qy * inv; r.z = qz * inv; r.w = qw * inv;
  return r;
}
__device__ __forceinline__ V3 rotate_point(Q4 q, V3 v) {  // :56-60
  const V3 qa = v3(q.x, q.y, q.z);
  return (2.0f * dot(qa, v)) * qa + (q.w * q.w - dot(qa, qa)) * v + (2.0f * q.w) * cross(qa, v);
}
__device__ __forceinline__ V3 sample_ggx_vndf(V3 Ve, float ax, float ay, V2 u) {  // :224-269 (Heitz)
  const V3 Vh = normalize(v3(ax * Ve.x, ay * Ve.y, Ve.z));
  const float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
  const V3 T1 = lensq > 0.0f ? v3(-Vh.y, Vh.x, 0.0f) * (1.0f / sqrtf(lensq)) : v3(1.0f, 0.0f, 0.0f);
  const V3 T2 = cross(Vh, T1);
  const float r = sqrtf(u.x);
  const float phi = (2.0f * kPi) * u.y;
  const float t1 = r * cr_cos(phi);
  float t2 = r * cr_sin(phi);
  const float s = 0.5f * (1.0f + Vh.z);
  t2 = lerpf(sqrtf(1.0f - t1 * t1), t2, s);
  const V3 Nh = t1 * T1 + t2 * T2 + sqrtf(smax(0.0f, 1.0f - t1 * t1 - t2 * t2)) * Vh;
  return normalize(v3(ax * Nh.x, ay * Nh.y, smax(0.0f, Nh.z)));
}
// evalIndirectCombinedBRDF :454-502.  type 1 = DIFFUSE_TYPE, 2 = SPECULAR_TYPE.  weight in/out.
__device__ __forceinline__ bool eval_indirect_brdf(V2 u, V3 N, V3 V, const Material& m, int type, V3& dir, V3& weight) {
  const Q4 q = rotation_to_z(N);
  const V3 Vl = rotate_point(q, V);
  const V3 Nl = v3(0.0f, 0.0f, 1.0f);
  V3 rl = v3(0.0f, 0.0f, 0.0f);
  if (type == 1) {
    const float a = sqrtf(u.x), b = (2.0f * kPi) * u.y;  // sampleHemisphere :62-76
    rl = v3(a * cr_cos(b), a * cr_sin(b), sqrtf(1.0f - u.x));
    const BrdfData d = prepare_brdf(Nl, rl, Vl, m);
    weight = d.diffR * 1.0f;  // lambertian() == 1
    const V3 Hs = sample_ggx_vndf(Vl, d.alpha, d.alpha, u);
    const float VdotH = smax(0.00001f, smin(1.0f, dot(Vl, Hs)));
    weight = weight * one_minus(fresnel_schlick(d.specF0, shadowed_f90(d.specF0), VdotH));
  } else if (type == 2) {
    // sampleSpecularMicrofacet :351-383 takes 'weight' by value: the caller's weight is untouched
    const BrdfData d = prepare_brdf(Nl, v3(0.0f, 0.0f, 1.0f), Vl, m);
    const V3 H = (d.alpha == 0.0f) ? v3(0.0f, 0.0f, 1.0f) : sample_ggx_vndf(Vl, d.alpha, d.alpha, u);
    rl = reflect(-Vl, H);
  }
  if (luminance(weight) == 0.0f) return false;
  Q4 qi;
  qi.x = -q.x; qi.y = -q.y; qi.z = -q.z; qi.w = q.w;
  dir = normalize(rotate_point(qi, rl));
  return true;
}
__device__ __forceinline__ float brdf_probability(const Material& m, V3 V, V3 N) {  // :504-526
  const float sF0 = luminance(specular_f0(m.base, m.metal));
  const float dR = luminance(diffuse_reflectance(m.base, m.metal));
  const float ff = smax(0.0f, dot(V, N));
  const V3 F0v = v3(sF0, sF0, sF0);
  const float fr = saturate(luminance(fresnel_schlick(F0v, shadowed_f90(F0v), ff)));
  const float adj = fr * 0.5f;
  const float spec = adj;
  const float diff = dR * (1.0f - adj) * 1.5f;
  const float p = spec / smax(0.0001f, (spec + diff));
  return clampf(p, 0.05f, 0.7f);
}

// ---- Scene queries
__device__ __forceinline__ V3 texel_color(uint32_t c) {  // Scene.cpp:225-229
  const float s = 1.0f / 255.0f;
  return v3((float)((c >> 16) & 0xFF) * s, (float)((c >> 8) & 0xFF) * s, (float)(c & 0xFF) * s);
}
__device__ __forceinline__ V3 texel_normal(uint32_t c) {  // :231-235
  const float s = 2.0f / 255.0f;
  return v3((float)((c >> 16) & 0xFF) * s - 1.0f, (float)((c >> 8) & 0xFF) * s - 1.0f, (float)(c & 0xFF) * s - 1.0f);
}
__device__ __forceinline__ float srgb1(float c) {  // :256-263
  return (c <= 0.04045f) ? (c / 12.92f) : cr_pow((c + 0.055f) / 1.055f, 2.4f);
}

struct HitAttr {
  V3 N;        // shading normal
  Material m;
  uint32_t kind;  // instance material kind (kMatDielectric takes Trace's dielectric branch)
};

// uv = v*uv2 + u*uv1 + w*uv0 (Scene.cpp:75-77,156-158); texel index with ALBEDO dims (:79-85,160-165)
__device__ __forceinline__ uint32_t texel_index(const TexDev& A, float2 uv) {
  const int iu = (int)(uv.x * (float)A.w) % A.w;
  const int iv = (int)(uv.y * (float)A.h) % A.h;
  return (uint32_t)(iu + iv * A.w);
}

__device__ __forceinline__ V3 geometry_normal(const SceneDev& S, uint32_t inst, uint32_t prim) {  // :47-58
  const InstDev& I = S.inst[inst];
  const MeshDev& M = S.mesh[I.mesh];
  const float4 f = reinterpret_cast<const float4*>(S.stri + M.prim_base + prim)[6];
  return xform_vector(v3(f.x, f.y, f.z), I.nrm);
}

__device__ __forceinline__ HitAttr hit_attributes(const SceneDev& S, uint32_t inst, uint32_t prim, float u, float v,
                                                  bool normalmapped) {
  HitAttr out;
  const InstDev& I = S.inst[inst];
  const MeshDev& M = S.mesh[I.mesh];
  const float4* st = reinterpret_cast<const float4*>(S.stri + M.prim_base + prim);
  const float w = 1.0f - u - v;
  const float4 s0 = st[0], s1 = st[1], s2 = st[2], s3 = st[3];  // n0 n1 n2 | uv0 uv1 uv2 | p0.x
  const float2 uv0 = make_float2(s2.y, s2.z), uv1 = make_float2(s2.w, s3.x), uv2 = make_float2(s3.y, s3.z);
  float2 uv;
  uv.x = v * uv2.x + u * uv1.x + w * uv0.x;
  uv.y = v * uv2.y + u * uv1.y + w * uv0.y;
  const TexDev A = S.tex[M.tex[0]];
  const uint32_t px = texel_index(A, uv);
  const V3 n0 = v3(s0.x, s0.y, s0.z), n1 = v3(s0.w, s1.x, s1.y), n2 = v3(s1.z, s1.w, s2.x);
  // ---- GetShadingNormal (:60-138)
  if (M.tex[1] >= 0 && normalmapped) {
    const V3 nc = texel_normal(S.texels[S.tex[M.tex[1]].offset + px]);
    const float4 s4 = st[4], s5 = st[5];  // p0.yz p1.xy | p1.z p2
    const V3 p0 = v3(s3.w, s4.x, s4.y), p1 = v3(s4.z, s4.w, s5.x), p2 = v3(s5.y, s5.z, s5.w);
    const V3 edge1 = p1 - p0, edge2 = p2 - p0;
    const float d1x = uv1.x - uv0.x, d1y = uv1.y - uv0.y, d2x = uv2.x - uv0.x, d2y = uv2.y - uv0.y;
    const float det = d1x * d2y - d1y * d2x;
    const float invDet = 1.0f / det;
    const V3 T = normalize(invDet * (d2y * edge1 - d1y * edge2));
    const V3 B = normalize(invDet * (-d2x * edge1 + d1x * edge2));
    V3 fn = v3(n0.x * w + n1.x * u + n2.x * v, n0.y * w + n1.y * u + n2.y * v, n0.z * w + n1.z * u + n2.z * v);
    fn = xform_vector(fn, I.nrm);
    const V3 N = normalize(fn);
    // glm: colorNorm * transpose(TBN)  (type_mat3x3.inl:477-483)
    out.N = normalize(v3(T.x * nc.x + B.x * nc.y + N.x * nc.z, T.y * nc.x + B.y * nc.y + N.y * nc.z,
                         T.z * nc.x + B.z * nc.y + N.z * nc.z));
  } else {
    const V3 it = v3(n0.x * w + n1.x * u + n2.x * v, n0.y * w + n1.y * u + n2.y * v, n0.z * w + n1.z * u + n2.z * v);
    out.N = xform_vector(it, I.nrm);  // not normalised (Scene.cpp:134-136)
  }
  // ---- GetMaterialBRDF (:140-218)
  const uint32_t ct = S.texels[A.offset + px];  // srgb1(texel_color(ct)) per channel, tabulated
  out.m.base = v3(S.srgb[(ct >> 16) & 0xFFu], S.srgb[(ct >> 8) & 0xFFu], S.srgb[ct & 0xFFu]);
  out.m.metal = 0.0f;
  out.m.rough = 0.0f;
  out.m.emis = v3(0.0f, 0.0f, 0.0f);
  if (M.tex[2] >= 0) {
    const uint32_t rma = S.texels[S.tex[M.tex[2]].offset + px];
    const float sc = 1.0f / 255.0f;
    out.m.rough = (float)((rma >> 8) & 255) * sc;
    out.m.metal = (float)(rma & 255) * sc;
  }
  if (M.tex[3] >= 0) out.m.emis = texel_color(S.texels[S.tex[M.tex[3]].offset + px]);
  out.kind = I.kind;
  if (I.kind == kMatMirror) {  // perfect mirror (:199-204): base colour kept, emission never set
    out.m.metal = 1.0f;
    out.m.rough = 0.0f;
    out.m.emis = v3(0.0f, 0.0f, 0.0f);
  }
  return out;
}

// Camera::SampleSkybox (Core/Camera.cpp:43-74)
__device__ __forceinline__ V3 sample_sky(const SceneDev& S, V3 D) {
  if (!S.sky) return v3(0.0f, 0.0f, 0.0f);
  const float u = 0.5f + (cr_atan2(D.z, D.x) / (2.0f * kPi));
  const float v = cr_acos(D.y) / kPi;
  const float uTex = u * (float)S.skyw, vTex = v * (float)S.skyh;
  const uint32_t W = (uint32_t)S.skyw, H = (uint32_t)S.skyh;
  const uint32_t u0 = (uint32_t)floorf(uTex) % W, v0 = (uint32_t)floorf(vTex) % H;
  const uint32_t u1 = (u0 + 1) % W, v1 = (v0 + 1) % H;
  const float du = uTex - (float)u0, dv = vTex - (float)v0;
  const uint32_t i00 = (u0 + v0 * W) * 3, i01 = (u1 + v0 * W) * 3, i10 = (u0 + v1 * W) * 3, i11 = (u1 + v1 * W) * 3;
  const float* P = S.sky;
  const V3 c00 = v3(P[i00], P[i00 + 1], P[i00 + 2]), c01 = v3(P[i01], P[i01 + 1], P[i01 + 2]);
  const V3 c10 = v3(P[i10], P[i10 + 1], P[i10 + 2]), c11 = v3(P[i11], P[i11 + 1], P[i11 + 2]);
  const V3 a = c00 + du * (c01 - c00);
  const V3 b = c10 + du * (c11 - c10);
  return a + dv * (b - a);
}

}  // namespace prt
