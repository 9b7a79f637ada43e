// prt_scene.h -- device-resident scene layout (HBM) shared by host and kernels.
//
//   nodes8  Node8[]    80 B each, all meshes' BLASes concatenated (bvh_build.h)
//   tris    TriMT[]    48 B each, leaf order, MT-ready {v0,prim | e1 | e2}
//   stri    ShadeTri[T] everything shading reads for one primitive in one 128-B line, prim order
//                       (global prim = mesh.prim_base + prim): Model::fixedNormals, fixedTextureCoords,
//                       the object-space corner positions vertices[indices[3p+k]], faceNormals
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
  uint32_t kind;   // instance material: kMatTextured / kMatDielectric / kMatMirror (Core/Scene.cpp:193-205)
};
enum : uint32_t { kMatTextured = 0, kMatDielectric = 1, kMatMirror = 2 };

// one primitive's shading inputs (Core/Scene.cpp:47-218 reads them from five arrays; here one line)
struct alignas(16) ShadeTri {
  float n[9];    // fixedNormals[3p..3p+2].xyz
  float uv[6];   // fixedTextureCoords[3p..3p+2]
  float p[9];    // vertices[indices[3p+k]], k = 0..2 (normal-map tangent frame, Scene.cpp:93-103)
  float fn[3];   // faceNormals[p]
  uint32_t pad[5];  // pad[0]: index of the primitive's TriMT record (leaf order)
};
static_assert(sizeof(ShadeTri) == 128, "ShadeTri must be one 128-byte line");

struct MeshDev {
  uint32_t root;       // Node8 index of the BLAS root
  uint32_t prim_base;  // offset into the per-triangle shading arrays
  uint32_t vert_base;  // unused (kept for layout)
  uint32_t tri_count;
  int32_t tex[4];      // albedo, normal, metalness, emission (-1 = none)
};

struct TexDev {
  uint32_t offset;
  int32_t w, h;
  int32_t pad;
};

// up to kLinearInstances instances are tested as a linear list of world boxes; above that (or with PRT_TLAS=1)
// the rays walk an 8-wide BVH over the instance boxes (the reference's TLAS, Core/tiny_bvh.h:2500-2565)
constexpr int kLinearInstances = 64;
constexpr int kMaxInstances = 1 << 24;

// one BLAS node (80 B, 5 x 16-B loads).  A 128-B stride (one line per node) measured slower: the footprint grows
// 1.6x and the L2 holds less of the tree
__host__ __device__ inline const uint4* blas_node(const Node8* base, uint32_t node) {
  return reinterpret_cast<const uint4*>(base + node);
}

struct SceneDev {
  const Node8* nodes8;    // all BLASes; MeshDev.root indexes it
  const TriMT* tris;
  const ShadeTri* stri;
  const uint32_t* texels;
  const TexDev* tex;
  const InstDev* inst;
  const MeshDev* mesh;
  const float* sky;
  const float* srgb;  // srgbToLinear(byte / 255) for byte 0..255
  const Node8* tlas8;          // instance BVH (root = node 0; bvh_build.h build_tlas8), when tlas != 0
  const uint32_t* tlas_slot;   // 8 per TLAS node: instance id of each leaf slot
  int32_t ninst;
  int32_t skyw, skyh;
  uint32_t pbits;   // prim bits of a packed hit word (prt_queue.h pack_hit)
  int32_t spill_levels;  // traversal stack levels beyond the LDS ones, in HBM (prt_traverse8.h LaneStack)
  uint2* spill;          // level-major spill columns (nullptr: the BVH fits the LDS stacks)
  uint32_t* diag;        // device diagnostics ([1]: kernarg layout check failed): [0] traversal stack overflows (a node group that found no stack
                         // level was dropped; the host sizes the stacks so this stays 0, prt_stats.stack_overflows)
  int32_t tlas;     // 1: rays walk tlas8 (more than kLinearInstances instances, or PRT_TLAS=1); 0: linear list
  // lights (Core/Renderer.cpp:216-310) and camera (Core/Camera.cpp:29-36)
  float ppos[12], pcol[12];
  float dpos[3], dcol[3], spos[3], scol[3], srot[3];
  float cam[12];  // pos, top_left, top_right, bottom_left
  // post-processing (Core/Camera.cpp:113-139): Panini primary rays when panini != 0
  float basis[9];  // right, up, ahead (Core/Camera.h:17)
  float pan_b, pan_d;
  int32_t panini;
  int32_t pad1;
  // extensions beyond the reference's Trace: one area light, dielectric instances
  float al[16];     // p0, eu, ev, n = normalize(cross(eu, ev)), Le, area
  int32_t area;     // 1 = the area light is set
  int32_t area_two_sided;
  int32_t has_diel; // some instance is kMatDielectric
  int32_t pad2;
};

}  // namespace prt
