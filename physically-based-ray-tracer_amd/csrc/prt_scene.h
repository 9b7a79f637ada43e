// prt_scene.h -- device-resident scene layout (HBM) shared by host and kernels.
//
//   nodes   Node4[]    128 B each, all meshes' BLASes concatenated (bvh_build.h)
//   tris    TriMT[]    48 B each, leaf order, MT-ready {v0,prim | e1 | e2}
//   fnrm    float4[3T] Model::fixedNormals, prim order (global prim = mesh.prim_base + prim)
//   fuv     float2[3T] Model::fixedTextureCoords
//   vidx    int32[3T]  Model::indices (mesh-local vertex ids)
//   vert    float[3V]  Model::vertices (global vertex = mesh.vert_base + id)
//   facen   float[3T]  Model::faceNormals
//   texels  uint32[]   every texture's 0x00RRGGBB pixels back to back
//   inst    InstDev[]  inverse transform (rays), inverse-transpose (normals), world AABB
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bvh_build.h"

namespace prt {

struct InstDev {
  float inv[16];   // BLASInstance::invTransform (Core/tiny_bvh.h:7883-7905)
  float nrm[16];   // mat4(transform).Inverted().Transposed() (Core/Scene.cpp:51-55)
  float bmin[3];   // world AABB of the BLAS root (BLASInstance::Update), inflated
  uint32_t mesh;
  float bmax[3];
  uint32_t pad;
};

struct MeshDev {
  uint32_t root;       // Node4 index of the BLAS root
  uint32_t prim_base;  // offset into the per-triangle shading arrays
  uint32_t vert_base;  // offset (in vertices) into vert
  uint32_t tri_count;
  int32_t tex[4];      // albedo, normal, metalness, emission (-1 = none)
};

struct TexDev {
  uint32_t offset;
  int32_t w, h;
  int32_t pad;
};

constexpr int kMaxInstances = 64;

struct SceneDev {
  const Node4* nodes;
  const Node8* nodes8;  // Node8 BLASes (layout 8); root indices in MeshDev.root refer to the active layout
  const TriMT* tris;
  const float4* fnrm;
  const float2* fuv;
  const int32_t* vidx;
  const float* vert;
  const float* facen;
  const uint32_t* texels;
  const TexDev* tex;
  const InstDev* inst;
  const MeshDev* mesh;
  const float* sky;
  int32_t ninst;
  int32_t skyw, skyh;
  int32_t pad0;
  // lights (Core/Renderer.cpp:216-310) and camera (Core/Camera.cpp:29-36)
  float ppos[12], pcol[12];
  float dpos[3], dcol[3], spos[3], scol[3], srot[3];
  float cam[12];  // pos, top_left, top_right, bottom_left
};

}  // namespace prt
