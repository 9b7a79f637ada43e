// prt_tlas.h -- the instance BVH refitted on the device (prt_tlas.hip): level order and launcher.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "prt_scene.h"

namespace prt {

// a host-built instance BVH's nodes grouped by depth, deepest level first (the order a bottom-up refit needs)
struct TlasTopo {
  std::vector<uint32_t> order;      // node indices, level by level
  std::vector<uint32_t> level_off;  // first entry of each level in order
  std::vector<uint32_t> level_cnt;  // nodes per level
};
TlasTopo tlas_topology(const std::vector<Node8>& nodes);
// the instance BVH's description on the device (instance counts up to kGpuSmallBuild): node count and the refit
// order's levels, deepest first (order[level_off[l] ..] holds level l's level_cnt[l] nodes).  valid = 0 marks a device
// rebuild that produced no usable tree (the commit then keeps the current one)
constexpr int kTlasMaxLevels = 64;
struct TlasMeta {
  uint32_t n_nodes, nlevels, valid, depth;
  uint32_t level_off[kTlasMaxLevels], level_cnt[kTlasMaxLevels];
};
TlasMeta tlas_meta(const TlasTopo& T, uint32_t n_nodes);
// sync-free device rebuild for n <= kGpuSmallBuild instances (bvh_gpu.h gpu_build_blas8_small), on stream s: the
// refit records' boxes (inst) -> back buffers nodes / slot / order / meta.  Scratch: fat 12 n floats, tris n TriMT,
// scratch gpu_small_scratch_bytes(n), out 4 + kTlasMaxLevels words.  depth_cap: the deepest tree the context's stacks
// are sized for (deeper: meta.valid = 0)
hipError_t gpu_rebuild_tlas_small(hipStream_t s, const InstDev* inst, int32_t n, float* fat, TriMT* tris,
                                  void* scratch, uint32_t* out, Node8* nodes, uint32_t* slot, uint32_t* order,
                                  TlasMeta* meta, int depth_cap);
// the back tree copied over the front one when valid (one workgroup, in the render stream's order)
hipError_t launch_tlas_commit(hipStream_t s, const TlasMeta* mb, const Node8* nb, const uint32_t* sb,
                              const uint32_t* ob, TlasMeta* mf, Node8* nf, uint32_t* sf, uint32_t* of,
                              uint32_t* rejected);
// the refit over the device meta's levels, one workgroup, one launch
hipError_t launch_tlas_refit_meta(hipStream_t s, const InstDev* inst, const TlasMeta* meta, const uint32_t* order,
                                  Node8* nodes, const uint32_t* slot, float* aabb);
// queue the refit on stream s over the refit instance records `inst` (their inflated world boxes): one launch per
// level; order_dev = T.order on the device; aabb: 6 floats per node of scratch; nothing is synchronised
// rebuild the instance BVH's topology on the device over the instances' inflated world boxes (boxes: 6 floats per
// instance, device): bvh_gpu.hip's PLOC + treelet restructuring + SAH-optimal collapse with one instance per leaf
// slot, converted to the instance form (slot[8j + s], tri_base 8j).  Scratch: fat 12 n floats, tris n TriMT; nodes:
// room for n Node8, slot 8 n.  Fills the refit order T (level by level, as the collapse emits), the depth and the
// node count.  Synchronises on s (only) once per builder level; its scratch is stream-ordered.
struct TriMT;
hipError_t gpu_build_tlas8(hipStream_t s, const float* boxes, int32_t n, float* fat, TriMT* tris, Node8* nodes,
                           uint32_t* slot, TlasTopo* T, int* depth, uint32_t* n_nodes);
// the tree's SAH cost over its current boxes (after a refit) into *out (device), one block
hipError_t launch_tlas_cost(hipStream_t s, const Node8* nodes, uint32_t n_nodes, const float* aabb,
                            const InstDev* inst, const uint32_t* slot, double* out, const TlasMeta* meta = nullptr);
hipError_t launch_tlas_refit(hipStream_t s, const InstDev* inst, const TlasTopo& T, const uint32_t* order_dev,
                             Node8* nodes, const uint32_t* slot, float* aabb);

}  // namespace prt
