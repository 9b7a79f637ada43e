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
// queue the refit on stream s over the refit instance records `inst` (their inflated world boxes): one launch per
// level; order_dev = T.order on the device; aabb: 6 floats per node of scratch; nothing is synchronised
hipError_t launch_tlas_refit(hipStream_t s, const InstDev* inst, const TlasTopo& T, const uint32_t* order_dev,
                             Node8* nodes, const uint32_t* slot, float* aabb);

}  // namespace prt
