// prt_math.h -- device-side float math with the reference's exact expression order.
//
// The whole product TU is compiled with -ffp-contract=off: every +,-,*,/ and sqrtf below is one
// IEEE-754 rounding (hipcc keeps f32 division and sqrt correctly rounded by default), so these
// functions reproduce the reference's C++ float expressions bit for bit.  Transcendentals the
// reference calls in float (std::pow, cos, sin, atan2f, acosf) are evaluated in double and rounded
// once to float: a correctly-rounded float libm, identical on CPU and GPU except for inputs whose
// double results straddle a float rounding boundary (~2^-29 per call).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PRT_HD __host__ __device__ __forceinline__

namespace prt {

constexpr float kEpsilon = 0.01f;           // template/common.h:26
constexpr float kFar = 1e30f;               // BVH_FAR, Core/tiny_bvh.h:131
constexpr float kPi = 3.141592653589f;      // PI macro, Core/BRDF.h:27
constexpr float kMinDielectricsF0 = 0.4f;   // Core/BRDF.h:65

struct V3 { float x, y, z; };
struct V2 { float x, y; };
struct Q4 { float x, y, z, w; };

PRT_HD V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
PRT_HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PRT_HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PRT_HD V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
PRT_HD V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
PRT_HD V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
PRT_HD V3 operator/(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
PRT_HD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
PRT_HD V3 one_minus(V3 a) { return v3(1.0f - a.x, 1.0f - a.y, 1.0f - a.z); }        // float3(1) - a
PRT_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }        // tmpl8math.h:495
PRT_HD V3 cross(V3 a, V3 b) {                                                      // tmpl8math.h:553
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
PRT_HD float length(V3 a) { return sqrtf(dot(a, a)); }
// tmpl8 / glm normalize: v * (1/sqrtf(dot(v,v)))  (tmpl8math.h:139,517; glm func_geometric.inl:104)
PRT_HD V3 normalize(V3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return v * inv; }
// tinybvh_normalize (Core/tiny_bvh.h:404-408)
PRT_HD V3 normalize_bvh(V3 a) {
  float l = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
  float rl = l == 0 ? 0 : (1.0f / l);
  return a * rl;
}
PRT_HD float safercp(float x) { return x > 1e-12f ? (1.0f / x) : (x < -1e-12f ? (1.0f / x) : kFar); }
// std::min / std::max (precomp.h:35 'using namespace std')
PRT_HD float smin(float a, float b) { return (b < a) ? b : a; }
PRT_HD float smax(float a, float b) { return (a < b) ? b : a; }
// tmpl8 fminf/fmaxf/clamp (tmpl8math.h:137-138,446), saturate (BRDF.h:163)
PRT_HD float tmin_(float a, float b) { return a < b ? a : b; }
PRT_HD float tmax_(float a, float b) { return a > b ? a : b; }
PRT_HD float clampf(float f, float a, float b) { return tmax_(a, tmin_(f, b)); }
PRT_HD float saturate(float x) { return clampf(x, 0.0f, 1.0f); }
PRT_HD V3 lerp(V3 a, V3 b, float t) { return a + t * (b - a); }                   // tmpl8math.h:470
PRT_HD float lerpf(float a, float b, float t) { return a + t * (b - a); }
PRT_HD V3 reflect(V3 i, V3 n) { return i - (2.0f * n) * dot(n, i); }              // tmpl8math.h:547

PRT_HD float cr_pow(float x, float y) { return (float)pow((double)x, (double)y); }
// pow(x, 5) (BRDF.cpp:84-87 Fresnel): x^5 in double (three roundings, <= 3 ulp of double) rounded once to
// float -- the correctly rounded float x^5 except within 2^-50 of a float rounding boundary; the oracle
// evaluates the identical double expression
PRT_HD float pow5(float x) {
  const double d = (double)x, d2 = d * d;
  return (float)(d2 * d2 * d);
}
PRT_HD float cr_sin(float x) { return (float)sin((double)x); }
PRT_HD float cr_cos(float x) { return (float)cos((double)x); }
PRT_HD float cr_atan2(float y, float x) { return (float)atan2((double)y, (double)x); }
PRT_HD float cr_acos(float x) { return (float)acos((double)x); }

// tinybvh_transform_point / _vector (Core/tiny_bvh.h:409-422); T row-major 4x4
PRT_HD V3 xform_point(V3 v, const float* T) {
  V3 r = v3(T[0] * v.x + T[1] * v.y + T[2] * v.z + T[3], T[4] * v.x + T[5] * v.y + T[6] * v.z + T[7],
            T[8] * v.x + T[9] * v.y + T[10] * v.z + T[11]);
  const float w = T[12] * v.x + T[13] * v.y + T[14] * v.z + T[15];
  if (w == 1) return r;
  return r * (1.f / w);
}
PRT_HD V3 xform_vector(V3 v, const float* T) {
  return v3(T[0] * v.x + T[1] * v.y + T[2] * v.z, T[4] * v.x + T[5] * v.y + T[6] * v.z,
            T[8] * v.x + T[9] * v.y + T[10] * v.z);
}

// ---- RNG: Marsaglia xorshift32 + WangHash seeding (template/tmpl8math.cpp:15-48)
PRT_HD uint32_t wang_hash(uint32_t s) {
  s = (s ^ 61) ^ (s >> 16);
  s *= 9;
  s = s ^ (s >> 4);
  s *= 0x27d4eb2du;
  s = s ^ (s >> 15);
  return s;
}
PRT_HD uint32_t init_seed(uint32_t base) {
  uint32_t s = wang_hash((base + 1) * 17);
  return s ? s : 0x12345678u;
}
PRT_HD float random_float(uint32_t& seed) {
  uint32_t s = seed;
  s ^= s << 13;
  s ^= s >> 17;
  s ^= s << 5;
  seed = s;
  return (float)s * 2.3283064365387e-10f;
}

}  // namespace prt
