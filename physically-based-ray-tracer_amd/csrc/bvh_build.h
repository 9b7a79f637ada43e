// bvh_build.h -- host-side BLAS builder producing the device layout.
//
// Replaces the reference's BVH8_CPU::BuildHQ chain (Core/tiny_bvh.h:4511-4519 -> BVH::BuildHQ
// :1968-2284 -> MBVH<8>::ConvertFrom :3706-3781 -> BVH8_CPU::ConvertFrom :4548-4680), which emits a
// CPU AVX2 layout.  Here: binned-SAH binary BVH over triangle bounds, collapsed to 4-wide nodes whose
// child bounds are stored SoA (one 128-byte node = one aligned 128-B line: 6 float4 child-bound
// vectors + int4 child refs) and a separate 48-byte-per-triangle Moeller-Trumbore record
// {v0,prim | e1 | e2} in leaf order, mirroring BVHTri4Leaf's precomputed edges (tiny_bvh.h:4614-4619).
#pragma once
#include <cstdint>
#include <vector>

namespace prt {

// child ref encoding
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kEmptyChild = 0xFFFFFFFFu;
inline uint32_t make_leaf(uint32_t first_tri, uint32_t count) { return kLeafBit | (first_tri << 2) | (count - 1); }

struct alignas(16) Node4 {
  float lox[4], hix[4], loy[4], hiy[4], loz[4], hiz[4];
  uint32_t child[4];
  uint32_t pad[4];
};
static_assert(sizeof(Node4) == 128, "Node4 must be one 128-byte line");

struct alignas(16) TriMT {
  float v0[3];
  uint32_t prim;   // mesh-local primitive index (tinybvh Intersection::prim)
  float e1[3];
  float pad1;
  float e2[3];
  float pad2;
};
static_assert(sizeof(TriMT) == 48, "TriMT must be 48 bytes");

struct BuiltBlas {
  std::vector<Node4> nodes;   // node 0 = root (always interior)
  std::vector<TriMT> tris;    // leaf order
  float bmin[3], bmax[3];     // root bounds (exact, not inflated)
  int depth = 0;
  int64_t leaves = 0;
};

// triangles: fat float4 x 3T (Model::triangles).  max_leaf <= 4.
BuiltBlas build_blas(const float* triangles, int32_t tri_count, int max_leaf = 4);

// ---- 8-wide compressed node (CWBVH-style, Ylitie et al. 2017 "Efficient Incoherent Ray Traversal on GPUs
// Through Compressed Wide BVHs"; own encoding).  80 bytes = 5 x 16-B loads per visit:
//   [0]  px py pz | ex ey ez imask      grid origin, per-axis power-of-two scale 2^(e-127), interior mask
//   [1]  child_base tri_base meta[8]    interior slot k -> child_base + popc(imask & ((1<<k)-1));
//                                       leaf slot k: meta = (tri offset << 3) | count (count 1..4)
//   [2-4] qlo{x,y,z}[8] qhi{x,y,z}[8]   child bounds quantised outward on the node grid
// Children sit in slots chosen per octant (slot s holds the child nearest for rays of octant s), so
// visiting slots in the order (i ^ ray_octant) is approximately front to back without sorting.
struct alignas(16) Node8 {
  float px, py, pz;
  uint8_t ex, ey, ez, imask;
  uint32_t child_base, tri_base;
  uint8_t meta[8];
  uint8_t qlox[8], qloy[8], qloz[8], qhix[8], qhiy[8], qhiz[8];
};
static_assert(sizeof(Node8) == 80, "Node8 must be 80 bytes");

struct BuiltBlas8 {
  std::vector<Node8> nodes;   // node 0 = root
  std::vector<TriMT> tris;    // grouped per node (leaf children's triangles contiguous)
  float bmin[3], bmax[3];
  int depth = 0;
  int64_t leaves = 0;
};
BuiltBlas8 build_blas8(const float* triangles, int32_t tri_count, int max_leaf = 3);

// ---- the same tree with fp16 child bounds on an 11-bit grid: 128 bytes = one aligned cache line.
//   [0]  px py pz | ex ey ez imask      as Node8 (grid step 2^(e-127), q in 0..2047)
//   [1]  child_base tri_base meta[8]    as Node8
//   [2-7] qlox qhix qloy qhiy qloz qhiz [8] fp16 integers; a ray loads the near/far block per axis by
//        its direction sign and feeds the halves straight into v_fma_mix_f32 (no conversions)
struct alignas(128) Node8H {
  float px, py, pz;
  uint8_t ex, ey, ez, imask;
  uint32_t child_base, tri_base;
  uint8_t meta[8];
  uint16_t qlox[8], qhix[8], qloy[8], qhiy[8], qloz[8], qhiz[8];
};
static_assert(sizeof(Node8H) == 128, "Node8H must be one 128-byte line");

struct BuiltBlas8H {
  std::vector<Node8H> nodes;
  std::vector<TriMT> tris;
  float bmin[3], bmax[3];
  int depth = 0;
  int64_t leaves = 0;
};
BuiltBlas8H build_blas8h(const float* triangles, int32_t tri_count, int max_leaf = 3);

// Same inflation rule the traversal relies on (see bvh_build.cpp).
void inflate_box(float* lo, float* hi);

}  // namespace prt
