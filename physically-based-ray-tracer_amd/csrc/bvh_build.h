// bvh_build.h -- host-side BLAS builder producing the device layout.
//
// Replaces the reference's BVH8_CPU::BuildHQ chain (Core/tiny_bvh.h:4511-4519 -> BVH::BuildHQ
// :1968-2284 -> MBVH<8>::ConvertFrom :3706-3781 -> BVH8_CPU::ConvertFrom :4548-4680), which emits a
// CPU AVX2 layout.  Here: binned-SAH binary BVH over triangle bounds, collapsed SAH-optimally into 8-wide
// quantised nodes (Node8, 80 B) plus a separate 48-byte-per-triangle Moeller-Trumbore record
// {v0,prim | e1 | e2} in leaf order, mirroring BVHTri4Leaf's precomputed edges (tiny_bvh.h:4614-4619).
#pragma once
#include <cstdint>
#include <vector>

namespace prt {

struct alignas(16) TriMT {
  float v0[3];
  uint32_t prim;   // mesh-local primitive index (tinybvh Intersection::prim)
  float e1[3];
  float pad1;
  float e2[3];
  float pad2;
};
static_assert(sizeof(TriMT) == 48, "TriMT must be 48 bytes");

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
// spatial: spatial-split binary build (SBVH, as the reference's BuildHQ) instead of binned object splits; a
// triangle may then be referenced by several leaves (tris holds one record per reference)
BuiltBlas8 build_blas8(const float* triangles, int32_t tri_count, int max_leaf = 3, bool spatial = false);

// ---- TLAS over instance world boxes (replaces BVH::Build over BLASInstances, Core/tiny_bvh.h:1732-1770): the same
// binned SAH + SAH-optimal 8-wide collapse with one instance per leaf slot.  A TLAS node's leaf slot s names its
// instance in slot[8 * node + s] (node.tri_base = 8 * node), so the traversal addresses an instance group like an
// interior group: base + slot.
struct BuiltTlas8 {
  std::vector<Node8> nodes;     // node 0 = root
  std::vector<uint32_t> slot;   // 8 per node: instance id of each leaf slot (0xFFFFFFFF elsewhere)
  int depth = 0;
  bool median = false;          // the SAH tree exceeded max_depth: the balanced median-split tree was built instead
};
// boxes: n x {lo[3], hi[3]} world AABBs (inflated).  max_depth > 0 (>= tlas8_median_depth(n)): a tree of at most
// that many levels (the SAH tree, or the median-split one when the SAH tree is deeper); at most max(n, 1) nodes
BuiltTlas8 build_tlas8(const float* boxes, int32_t n, int max_depth = 0);
int tlas8_median_depth(int32_t n);  // levels of the median-split instance BVH over n instances: ceil(ceil(log2 n) / 3)

// Same inflation rule the traversal relies on (see bvh_build.cpp).
void inflate_box(float* lo, float* hi);

}  // namespace prt
