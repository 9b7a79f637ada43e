// prt_tlas.hip -- the instance BVH (TLAS) refitted on the device, in stream order right after k_refit.
//
// The reference rebuilds its TLAS every frame after physics moved the game objects (Core/Renderer.cpp:33-41:
// BVH::Build over the BLASInstances' world boxes, Core/tiny_bvh.h:1732-1770).  Here the host SAH builder
// (bvh_build.cpp build_tlas8) rebuilds it for every prt_set_instances; above kHostSyncBuild instances that build runs
// on a worker thread (prt_api.cpp ensure_instances), and until it is committed every update queues, behind the refit
// of the instance records (prt_refit.h), one launch per tree level, deepest first: each node re-quantises its
// children's current boxes (the instances' inflated world boxes, or the boxes its child nodes just wrote) onto a fresh
// grid exactly as the host builder does (build_wide8: same inflation, grid exponent and outward rounding).  Which
// child sits in which slot only steers the traversal order; hits never depend on it (order-independent hit rule,
// conservative boxes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "bvh_build.h"
#include "prt_tlas.h"

namespace prt {
namespace {

// bvh_build.cpp inflate_box, in the same float operations
__device__ __forceinline__ void inflate(float* lo, float* hi) {
  for (int k = 0; k < 3; k++) {
    const float ext = fmaxf(fabsf(lo[k]), fabsf(hi[k]));
    const float pad = ext * 1e-6f + 1e-7f;
    lo[k] -= pad;
    hi[k] += pad;
  }
}
// bvh_build.cpp grid_exponent with qmax = 255
__device__ __forceinline__ uint32_t grid_exp(double ext) {
  if (!(ext > 0)) return 1;
  int e = (int)ceil(log2(ext / 255.0));
  while (ldexp(255.0, e) < ext) e++;
  while (e > -126 && ldexp(255.0, e - 1) >= ext) e--;
  return (uint32_t)min(254, max(1, e + 127));
}

// refit of one node: its interior children (one level deeper) were refitted before and left their boxes in aabb
__device__ __forceinline__ void refit_node(const InstDev* __restrict__ inst, uint32_t node, Node8* __restrict__ nodes,
                                           const uint32_t* __restrict__ slot, float* __restrict__ aabb) {
  Node8 nd = nodes[node];
  float clo[8][3], chi[8][3];
  bool used[8];
  float nlo[3] = {1e30f, 1e30f, 1e30f}, nhi[3] = {-1e30f, -1e30f, -1e30f};
  for (uint32_t s = 0; s < 8; s++) {
    used[s] = true;
    if ((nd.imask >> s) & 1u) {
      const float* b = aabb + 6 * (size_t)(nd.child_base + (uint32_t)__popc(nd.imask & ((1u << s) - 1u)));
      for (int a = 0; a < 3; a++) { clo[s][a] = b[a]; chi[s][a] = b[3 + a]; }
    } else if (slot[8 * (size_t)node + s] != 0xFFFFFFFFu) {
      const InstDev& I = inst[slot[8 * (size_t)node + s]];
      for (int a = 0; a < 3; a++) { clo[s][a] = I.bmin[a]; chi[s][a] = I.bmax[a]; }
    } else {
      used[s] = false;
      continue;
    }
    inflate(clo[s], chi[s]);
    for (int a = 0; a < 3; a++) { nlo[a] = fminf(nlo[a], clo[s][a]); nhi[a] = fmaxf(nhi[a], chi[s][a]); }
  }
  nd.px = nlo[0]; nd.py = nlo[1]; nd.pz = nlo[2];
  const double p[3] = {(double)nlo[0], (double)nlo[1], (double)nlo[2]};
  uint32_t e[3];
  for (int a = 0; a < 3; a++) e[a] = grid_exp((double)nhi[a] - p[a]);
  nd.ex = (uint8_t)e[0]; nd.ey = (uint8_t)e[1]; nd.ez = (uint8_t)e[2];
  // the grid step 2^(e - 127)'s exact inverse: the products are the quotients bit for bit (no double division)
  const double isc[3] = {ldexp(1.0, 127 - (int)e[0]), ldexp(1.0, 127 - (int)e[1]), ldexp(1.0, 127 - (int)e[2])};
  uint8_t* ql[3] = {nd.qlox, nd.qloy, nd.qloz};
  uint8_t* qh[3] = {nd.qhix, nd.qhiy, nd.qhiz};
  for (uint32_t s = 0; s < 8; s++) {
    for (int a = 0; a < 3; a++) {
      if (used[s]) {
        ql[a][s] = (uint8_t)fmin(255.0, fmax(0.0, floor(((double)clo[s][a] - p[a]) * isc[a])));
        qh[a][s] = (uint8_t)fmin(255.0, fmax(0.0, ceil(((double)chi[s][a] - p[a]) * isc[a])));
      } else {  // empty slot: an inverted box never hits
        ql[a][s] = 255;
        qh[a][s] = 0;
      }
    }
  }
  nodes[node] = nd;
  float* b = aabb + 6 * (size_t)node;
  for (int a = 0; a < 3; a++) { b[a] = nlo[a]; b[3 + a] = nhi[a]; }
}

// one level of the refit: the nodes order[0..count) (all at one depth)
__global__ void k_tlas_refit(const InstDev* __restrict__ inst, const uint32_t* __restrict__ order, uint32_t count,
                             Node8* __restrict__ nodes, const uint32_t* __restrict__ slot, float* __restrict__ aabb) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= count) return;
  refit_node(inst, order[j], nodes, slot, aabb);
}

}  // namespace

TlasTopo tlas_topology(const std::vector<Node8>& nodes) {
  // depth of every node from the root (node 0): interior children sit at child_base + rank among the interior slots
  std::vector<int32_t> depth(nodes.size(), -1);
  std::vector<uint32_t> stack{0};
  depth[0] = 0;
  int32_t maxd = 0;
  while (!stack.empty()) {
    const uint32_t n = stack.back();
    stack.pop_back();
    const Node8& nd = nodes[n];
    for (uint32_t s = 0, r = 0; s < 8; s++)
      if ((nd.imask >> s) & 1u) {
        const uint32_t c = nd.child_base + r++;
        depth[c] = depth[n] + 1;
        maxd = std::max(maxd, depth[c]);
        stack.push_back(c);
      }
  }
  TlasTopo T;
  for (int32_t d = maxd; d >= 0; d--) {  // deepest level first
    T.level_off.push_back((uint32_t)T.order.size());
    for (size_t n = 0; n < nodes.size(); n++)
      if (depth[n] == d) T.order.push_back((uint32_t)n);
    T.level_cnt.push_back((uint32_t)T.order.size() - T.level_off.back());
  }
  return T;
}

hipError_t launch_tlas_refit(hipStream_t s, const InstDev* inst, const TlasTopo& T, const uint32_t* order_dev,
                             Node8* nodes, const uint32_t* slot, float* aabb) {
  for (size_t l = 0; l < T.level_cnt.size(); l++) {
    const uint32_t cnt = T.level_cnt[l];
    hipLaunchKernelGGL(k_tlas_refit, dim3((cnt + 63) / 64), dim3(64), 0, s, inst, order_dev + T.level_off[l], cnt, nodes,
                       slot, aabb);
  }
  return hipGetLastError();
}

}  // namespace prt
