// prt_refit.h -- instance refit (the TLAS of this build): BLASInstance::Update per instance, host or device.
//
// The reference rebuilds its TLAS every frame after physics moved the game objects (Core/Renderer.cpp:33-41,
// Core/GameObject.cpp:53-67, BLASInstance::Update Core/tiny_bvh.h:7868-7905).  Here an instance is
// {inverse, inverse-transpose, conservative world box}; prt_set_instances ships the raw transforms and
// k_refit recomputes these on the device, in stream order with the frames that read them.
#pragma once
#include "prt_math.h"
#include "prt_scene.h"

namespace prt {

// what the host hands the refit per instance: BLASInstance::transform (row-major) + the BLAS root box
struct InstSrc {
  float T[16];
  float bmin[3];
  uint32_t mesh;
  float bmax[3];
  uint32_t kind;
};

// MESA 4x4 inverse (template/tmpl8math.h:701-746 == BLASInstance::InvertTransform, tiny_bvh.h:7883-7905)
PRT_HD void mesa_inverse(const float* c, float* out) {
  float inv[16];
  inv[0] = c[5] * c[10] * c[15] - c[5] * c[11] * c[14] - c[9] * c[6] * c[15] + c[9] * c[7] * c[14] + c[13] * c[6] * c[11] - c[13] * c[7] * c[10];
  inv[1] = -c[1] * c[10] * c[15] + c[1] * c[11] * c[14] + c[9] * c[2] * c[15] - c[9] * c[3] * c[14] - c[13] * c[2] * c[11] + c[13] * c[3] * c[10];
  inv[2] = c[1] * c[6] * c[15] - c[1] * c[7] * c[14] - c[5] * c[2] * c[15] + c[5] * c[3] * c[14] + c[13] * c[2] * c[7] - c[13] * c[3] * c[6];
  inv[3] = -c[1] * c[6] * c[11] + c[1] * c[7] * c[10] + c[5] * c[2] * c[11] - c[5] * c[3] * c[10] - c[9] * c[2] * c[7] + c[9] * c[3] * c[6];
  inv[4] = -c[4] * c[10] * c[15] + c[4] * c[11] * c[14] + c[8] * c[6] * c[15] - c[8] * c[7] * c[14] - c[12] * c[6] * c[11] + c[12] * c[7] * c[10];
  inv[5] = c[0] * c[10] * c[15] - c[0] * c[11] * c[14] - c[8] * c[2] * c[15] + c[8] * c[3] * c[14] + c[12] * c[2] * c[11] - c[12] * c[3] * c[10];
  inv[6] = -c[0] * c[6] * c[15] + c[0] * c[7] * c[14] + c[4] * c[2] * c[15] - c[4] * c[3] * c[14] - c[12] * c[2] * c[7] + c[12] * c[3] * c[6];
  inv[7] = c[0] * c[6] * c[11] - c[0] * c[7] * c[10] - c[4] * c[2] * c[11] + c[4] * c[3] * c[10] + c[8] * c[2] * c[7] - c[8] * c[3] * c[6];
  inv[8] = c[4] * c[9] * c[15] - c[4] * c[11] * c[13] - c[8] * c[5] * c[15] + c[8] * c[7] * c[13] + c[12] * c[5] * c[11] - c[12] * c[7] * c[9];
  inv[9] = -c[0] * c[9] * c[15] + c[0] * c[11] * c[13] + c[8] * c[1] * c[15] - c[8] * c[3] * c[13] - c[12] * c[1] * c[11] + c[12] * c[3] * c[9];
  inv[10] = c[0] * c[5] * c[15] - c[0] * c[7] * c[13] - c[4] * c[1] * c[15] + c[4] * c[3] * c[13] + c[12] * c[1] * c[7] - c[12] * c[3] * c[5];
  inv[11] = -c[0] * c[5] * c[11] + c[0] * c[7] * c[9] + c[4] * c[1] * c[11] - c[4] * c[3] * c[9] - c[8] * c[1] * c[7] + c[8] * c[3] * c[5];
  inv[12] = -c[4] * c[9] * c[14] + c[4] * c[10] * c[13] + c[8] * c[5] * c[14] - c[8] * c[6] * c[13] - c[12] * c[5] * c[10] + c[12] * c[6] * c[9];
  inv[13] = c[0] * c[9] * c[14] - c[0] * c[10] * c[13] - c[8] * c[1] * c[14] + c[8] * c[2] * c[13] + c[12] * c[1] * c[10] - c[12] * c[2] * c[9];
  inv[14] = -c[0] * c[5] * c[14] + c[0] * c[6] * c[13] + c[4] * c[1] * c[14] - c[4] * c[2] * c[13] - c[12] * c[1] * c[6] + c[12] * c[2] * c[5];
  inv[15] = c[0] * c[5] * c[10] - c[0] * c[6] * c[9] - c[4] * c[1] * c[10] + c[4] * c[2] * c[9] + c[8] * c[1] * c[6] - c[8] * c[2] * c[5];
  const float det = c[0] * inv[0] + c[1] * inv[4] + c[2] * inv[8] + c[3] * inv[12];
  if (det != 0) {
    const float invdet = 1.0f / det;
    for (int i = 0; i < 16; i++) out[i] = inv[i] * invdet;
  } else {
    for (int i = 0; i < 16; i++) out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
  }
}

// BLASInstance::Update: inverse, the normal matrix mat4(transform).Inverted().Transposed() (Core/Scene.cpp:
// 51-55) and the world box of the 8 transformed root corners, inflated so the TLAS test stays conservative
PRT_HD void refit_instance(const InstSrc& s, InstDev& I) {
  mesa_inverse(s.T, I.inv);
  for (int r = 0; r < 4; r++)
    for (int k = 0; k < 4; k++) I.nrm[4 * r + k] = I.inv[4 * k + r];
  I.mesh = s.mesh;
  I.kind = s.kind;
  const float* T = s.T;
  float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
  for (int j = 0; j < 8; j++) {
    const float p[3] = {j & 1 ? s.bmax[0] : s.bmin[0], j & 2 ? s.bmax[1] : s.bmin[1], j & 4 ? s.bmax[2] : s.bmin[2]};
    float t[3];
    for (int r = 0; r < 3; r++) t[r] = T[4 * r] * p[0] + T[4 * r + 1] * p[1] + T[4 * r + 2] * p[2] + T[4 * r + 3];
    const float w = T[12] * p[0] + T[13] * p[1] + T[14] * p[2] + T[15];
    if (w != 1)
      for (int r = 0; r < 3; r++) t[r] = t[r] * (1.f / w);
    for (int r = 0; r < 3; r++) {
      lo[r] = smin(lo[r], t[r]);
      hi[r] = smax(hi[r], t[r]);
    }
  }
  for (int r = 0; r < 3; r++) {
    const float ext = smax(fabsf(lo[r]), fabsf(hi[r]));
    const float pad = ext * 1e-5f + 1e-6f;
    I.bmin[r] = lo[r] - pad;
    I.bmax[r] = hi[r] + pad;
  }
}

}  // namespace prt
