// prt_post.h -- post-processing math shared by host and device: the Panini projection of
// Camera::GetPrimaryRay (Core/Camera.cpp:81-139) and the screen pass of Renderer::Tick
// (Core/Renderer.cpp:107-133).  float arithmetic in the reference's order; cos / sin / pow in double
// rounded once (the convention of prt_math.h, mirrored by oracle/prt_oracle.c).
#pragma once
#include "prt_math.h"

namespace prt {

// Camera::Panini's horizontal scale b (:86-93); depends on fov and distortion only, so the host
// evaluates it once per render call
PRT_HD float panini_scale(float fov, float distortion) {
  const float fo = kPi / 2 - fov * 0.5f;
  const float f = cr_cos(fo) / cr_sin(fo) * 2.0f;
  const float f2 = f * f;
  const float d2 = distortion * distortion;
  return (sqrtf(smax(0.0f, (distortion + d2) * (distortion + d2) * (f2 + f2 * f2))) - (distortion * f + f)) /
         (d2 + d2 * f2 - 1.0f);
}

// Camera::Panini (:94-110) for ndc already known; b = panini_scale(fov, distortion)
PRT_HD V3 panini_dir(float ndcx, float ndcy, float b, float distortion) {
  ndcx *= b;
  ndcy *= b;
  const float h = ndcx, v = ndcy;
  const float h2 = h * h;
  const float k = h2 / ((distortion + 1.0f) * (distortion + 1.0f));
  const float k2 = k * k;
  const float d2 = distortion * distortion;
  const float discr = smax(0.0f, k2 * d2 - (k + 1.0f) * (k * d2 - 1.0f));
  const float cosPhi = (-k * distortion + sqrtf(discr)) / (k + 1.0f);
  const float S = (distortion + 1.0f) / (distortion + cosPhi);
  const float tanTheta = v / S;
  float sinPhi = sqrtf(smax(0.0f, 1.0f - cosPhi * cosPhi));
  if (ndcx < 0.0f) sinPhi *= -1.0f;
  const float s = 1.0f / sqrtf(1.0f + tanTheta * tanTheta);
  return v3(sinPhi, tanTheta, cosPhi) * s;
}

// screen pass parameters (Core/Camera.h:11-31)
struct PostDev {
  float grade[4];
  float vig_int, vig_rad;
  int32_t aberration;
  int32_t W, H;
};

// the vignette factor of pixel (x, y) (:121-125)
PRT_HD float vignette(const PostDev& P, int32_t x, int32_t y) {
  float ux = (float)x / (float)P.W, uy = (float)y / (float)P.H;
  ux *= 1.0f - ux;
  uy *= 1.0f - uy;
  const float vig = ux * uy * P.vig_int;
  return cr_pow(vig, P.vig_rad);
}

}  // namespace prt
