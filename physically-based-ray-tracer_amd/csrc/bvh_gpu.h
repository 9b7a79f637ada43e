// bvh_gpu.h -- on-device BLAS build (bvh_gpu.hip): LBVH or PLOC + SAH-optimal 8-wide collapse into Node8 / TriMT.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "prt_scene.h"

namespace prt {

struct GpuBlasInfo {
  uint32_t nodes;   // Node8 written (node 0 = root)
  uint32_t tris;    // TriMT written (== triangle count)
  uint32_t leaves;  // leaf children
  int32_t depth;    // wide-tree levels
  float bmin[3], bmax[3];  // exact root bounds
};

// tri_dev: fat triangles float4 x 3T in device memory.  nodes_out: room for T Node8; tris_out: T TriMT.
// Synchronises on stream s once per tree level.  Child / triangle offsets are relative to the mesh.
// ploc: PLOC clustering (bvh_gpu.hip) instead of the LBVH radix tree for the binary tree.  level_ends (optional):
// the wide tree is emitted level by level, so level d's nodes are [level_ends[d-1], level_ends[d]) (level 0: [0, 1))
hipError_t gpu_build_blas8(hipStream_t s, const float* tri_dev, int32_t n_tris, int max_leaf, Node8* nodes_out,
                           TriMT* tris_out, GpuBlasInfo* info, bool ploc = false,
                           std::vector<uint32_t>* level_ends = nullptr, int trbvh = -1,  // trbvh < 0: PRT_TRBVH / default
                           int ploc_radius = 64);  // PLOC search radius: 64 (PRT_PLOC_R) or 512
// rebase a mesh's nodes into the concatenated arrays (in place) and record ShadeTri.pad[0] for its primitives
hipError_t gpu_blas_finish(hipStream_t s, Node8* nodes, uint32_t n_nodes, uint32_t node_base, const TriMT* tris,
                           uint32_t n_tris, uint32_t tri_base, ShadeTri* stri, uint32_t prim_base);

}  // namespace prt
