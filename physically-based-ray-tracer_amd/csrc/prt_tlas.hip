#include <cstdio>
#include <cstdlib>
// prt_tlas.hip -- the instance BVH (TLAS) refitted on the device, in stream order right after k_refit.
//
// The reference rebuilds its TLAS every frame after physics moved the game objects (Core/Renderer.cpp:33-41:
// BVH::Build over the BLASInstances' world boxes, Core/tiny_bvh.h:1732-1770).  Here the tree's topology (which
// instance or child node sits in which slot of which node) is built by the host SAH builder only when the set of
// instances changes (bvh_build.cpp build_tlas8); every prt_set_instances that keeps the instance count queues,
// behind the refit of the instance records (prt_refit.h), one launch per tree level, deepest first: each node
// re-quantises its children's current boxes (the instances' inflated world boxes, or the boxes its child nodes
// just wrote) onto a fresh grid exactly as the host builder does (build_wide8: same inflation, grid exponent and
// outward rounding).  No host BVH work and no synchronisation per frame.  Which child sits in which slot only
// steers the traversal order; hits never depend on it (order-independent hit rule, conservative boxes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "bvh_build.h"
#include "bvh_gpu.h"
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

// the whole refit in one workgroup, levels from the device-resident TlasMeta (deepest first) behind barriers
__global__ void __launch_bounds__(1024) k_tlas_refit_meta(const InstDev* __restrict__ inst,
                                                          const TlasMeta* __restrict__ meta,
                                                          const uint32_t* __restrict__ order, Node8* __restrict__ nodes,
                                                          const uint32_t* __restrict__ slot, float* __restrict__ aabb) {
  const uint32_t nl = meta->nlevels;
  for (uint32_t l = 0; l < nl && l < (uint32_t)kTlasMaxLevels; l++) {
    const uint32_t off = meta->level_off[l], cnt = meta->level_cnt[l];
    for (uint32_t j = threadIdx.x; j < cnt; j += blockDim.x) refit_node(inst, order[off + j], nodes, slot, aabb);
    __syncthreads();
  }
}

// ---- device rebuild of the topology: the instances' current world boxes through the device BLAS
// builder (bvh_gpu.hip: PLOC + SAH-optimal 8-wide collapse, one instance per leaf slot), converted to the
// instance-BVH form exactly as the host's build_tlas8 converts its BLAS-form tree

// instance i's inflated world box (6 floats) as the degenerate "triangle" {lo, hi, lo} (bvh_build.cpp build_tlas8)
__global__ void k_inst_fat(const float* __restrict__ boxes, int32_t n, float4* __restrict__ fat) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* b = boxes + 6 * (size_t)i;
  const float4 lo = make_float4(b[0], b[1], b[2], 0.0f), hi = make_float4(b[3], b[4], b[5], 0.0f);
  fat[3 * (size_t)i] = lo;
  fat[3 * (size_t)i + 1] = hi;
  fat[3 * (size_t)i + 2] = lo;
}

// the refit records' world boxes (InstDev bmin / bmax: refit_instance's inflated box, the boxes the host build reads)
// as degenerate triangles
__global__ void k_inst_fat_dev(const InstDev* __restrict__ inst, int32_t n, float4* __restrict__ fat) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const InstDev& I = inst[i];
  const float4 lo = make_float4(I.bmin[0], I.bmin[1], I.bmin[2], 0.0f), hi = make_float4(I.bmax[0], I.bmax[1], I.bmax[2], 0.0f);
  fat[3 * (size_t)i] = lo;
  fat[3 * (size_t)i + 1] = hi;
  fat[3 * (size_t)i + 2] = lo;
}

// the render stream's side of a device rebuild: the back tree replaces the front one when it is valid (the front
// tree is only ever written in render-stream order, so queued frames never see a half-written tree)
__global__ void __launch_bounds__(1024) k_tlas_commit(const TlasMeta* __restrict__ mb, const Node8* __restrict__ nb,
                                                      const uint32_t* __restrict__ sb, const uint32_t* __restrict__ ob,
                                                      TlasMeta* __restrict__ mf, Node8* __restrict__ nf,
                                                      uint32_t* __restrict__ sf, uint32_t* __restrict__ of,
                                                      uint32_t* __restrict__ rejected) {
  if (!mb->valid) {  // deeper than the stacks were sized for (or a failed build): the current tree stays
    if (threadIdx.x == 0) atomicAdd(rejected, 1u);
    return;
  }
  const uint32_t nn = mb->n_nodes;
  const uint4* ns = reinterpret_cast<const uint4*>(nb);
  uint4* nd = reinterpret_cast<uint4*>(nf);
  for (uint32_t i = threadIdx.x; i < 5u * nn; i += blockDim.x) nd[i] = ns[i];
  for (uint32_t i = threadIdx.x; i < 8u * nn; i += blockDim.x) sf[i] = sb[i];
  for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) of[i] = ob[i];
  const uint32_t* ms = reinterpret_cast<const uint32_t*>(mb);
  uint32_t* md = reinterpret_cast<uint32_t*>(mf);
  for (uint32_t i = threadIdx.x; i < sizeof(TlasMeta) / 4; i += blockDim.x) md[i] = ms[i];
}

// leaf slot s of node j -> the instance it holds (slot[8j + s]); tri_base = 8j (build_tlas8's conversion)
__global__ void k_tlas_slots(Node8* __restrict__ nodes, uint32_t n_nodes, const TriMT* __restrict__ tris,
                             uint32_t* __restrict__ slot) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n_nodes) return;
  Node8& nd = nodes[j];
  for (uint32_t s = 0; s < 8; s++)
    slot[8 * (size_t)j + s] = (!((nd.imask >> s) & 1u) && nd.meta[s]) ? tris[nd.tri_base + (nd.meta[s] >> 3)].prim
                                                                        : 0xFFFFFFFFu;
  nd.tri_base = 8u * j;
}

__device__ __forceinline__ double box_area(const float* lo, const float* hi) {
  const double dx = (double)hi[0] - lo[0], dy = (double)hi[1] - lo[1], dz = (double)hi[2] - lo[2];
  return (dx < 0 || dy < 0 || dz < 0) ? 0.0 : 2.0 * (dx * dy + dy * dz + dz * dx);
}
// the tree's node-visit SAH cost (the sum of its nodes' areas per unit root area) over the boxes the last refit left
// in aabb: one block
__global__ void __launch_bounds__(1024) k_tlas_cost(const Node8* __restrict__ nodes, uint32_t n_nodes,
                                                    const float* __restrict__ aabb, const InstDev* __restrict__ inst,
                                                    const uint32_t* __restrict__ slot, double* __restrict__ out,
                                                    const TlasMeta* __restrict__ meta) {
  __shared__ double red[1024];
  if (meta) n_nodes = meta->n_nodes;
  // the interior nodes' areas only: the leaf term (the instances' own boxes) does not change as instances move, so
  // it would dilute the growth the refit causes
  double acc = 0.0;
  for (uint32_t j = threadIdx.x; j < n_nodes; j += blockDim.x) {
    const float* b = aabb + 6 * (size_t)j;
    acc += box_area(b, b + 3);
  }
  (void)inst;
  (void)slot;
  red[threadIdx.x] = acc;
  __syncthreads();
  for (uint32_t w = blockDim.x / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double root = box_area(aabb, aabb + 3);
    out[0] = root > 0 ? red[0] / root : 0.0;
  }
}

}  // namespace

hipError_t gpu_build_tlas8(hipStream_t s, const float* boxes, int32_t n, float* fat, TriMT* tris, Node8* nodes,
                           uint32_t* slot, TlasTopo* T, int* depth, uint32_t* n_nodes) {
  if (n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_inst_fat, dim3((n + 255) / 256), dim3(256), 0, s, boxes, n, reinterpret_cast<float4*>(fat));
  GpuBlasInfo gi{};
  std::vector<uint32_t> ends;
  // PLOC search radius (PRT_TLAS_PLOC_R: 64 or 512, default 512) and treelet restructuring passes over its tree
  // (PRT_TLAS_TRBVH, default 0).  Measured on the 1,000-instance drift (scripts/tlas_drift.py): radius 64 without
  // restructuring renders 3-4 % behind a fresh host SAH tree, one pass 1-5 % behind at ~4 ms more per build
  const char* te = std::getenv("PRT_TLAS_TRBVH");
  const char* tr = std::getenv("PRT_TLAS_PLOC_R");
  hipError_t e = gpu_build_blas8(s, fat, n, 1, nodes, tris, &gi, true, &ends, te ? std::max(0, std::atoi(te)) : 0,
                                 tr ? std::atoi(tr) : 512);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_tlas_slots, dim3((gi.nodes + 255) / 256), dim3(256), 0, s, nodes, gi.nodes, tris, slot);
  // the collapse emits level by level: the refit order is the identity, levels deepest first
  T->order.resize(gi.nodes);
  for (uint32_t i = 0; i < gi.nodes; i++) T->order[i] = i;
  T->level_off.clear();
  T->level_cnt.clear();
  for (size_t l = ends.size(); l-- > 0;) {
    const uint32_t b = l == 0 ? 0u : ends[l - 1];
    T->level_off.push_back(b);
    T->level_cnt.push_back(ends[l] - b);
  }
  *depth = gi.depth;
  *n_nodes = gi.nodes;
  return hipGetLastError();
}

// the one-workgroup kernels around a device rebuild run beside the persistent traversal, which leaves no VGPRs free
// on a SIMD it holds: a 4-wave workgroup finds room as soon as a few traversal waves have exited, a 16-wave one
// waits for a whole CU to drain
constexpr int kTlasSmallThreads = 256;

hipError_t launch_tlas_cost(hipStream_t s, const Node8* nodes, uint32_t n_nodes, const float* aabb,
                            const InstDev* inst, const uint32_t* slot, double* out, const TlasMeta* meta) {
  hipLaunchKernelGGL(k_tlas_cost, dim3(1), dim3(1024), 0, s, nodes, n_nodes, aabb, inst, slot, out, meta);
  return hipGetLastError();
}

hipError_t gpu_rebuild_tlas_small(hipStream_t s, const InstDev* inst, int32_t n, float* fat, TriMT* tris,
                                  void* scratch, uint32_t* out, Node8* nodes, uint32_t* slot, uint32_t* order,
                                  TlasMeta* meta, int depth_cap) {
  if (n <= 0 || n > kGpuSmallBuild) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_inst_fat_dev, dim3((n + 255) / 256), dim3(256), 0, s, inst, n, reinterpret_cast<float4*>(fat));
  // PLOC search radius of the single-workgroup build (PRT_TLAS_SMALL_R, default 64: bvh_gpu.hip kSmallR)
  const char* re = std::getenv("PRT_TLAS_SMALL_R");
  static_assert(sizeof(TlasMeta) == 4 * (4 + 2 * kTlasMaxLevels), "TlasMeta words (the collapse launch writes them)");
  SmallTlasOut to;
  to.slot = slot;
  to.order = order;
  to.meta = reinterpret_cast<uint32_t*>(meta);
  to.depth_cap = (uint32_t)depth_cap;
  const hipError_t e = gpu_build_blas8_small(s, fat, n, 1, nodes, tris, scratch, out, out + 4, kTlasMaxLevels,
                                             re ? std::atoi(re) : 0, to);
  if (e != hipSuccess) return e;
  if (std::getenv("PRT_TLAS_SMALL_TIMES")) {  // diagnostic: the build's phase clock (waits for the side stream)
    uint32_t w[64];
    if (hipMemcpyAsync(w, gpu_small_ctr(scratch, n), sizeof(w), hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess) {
      auto t = [&](int k) { return (double)(((unsigned long long)w[9 + 2 * k] << 32) | w[8 + 2 * k]) / 100.0; };
      std::fprintf(stderr, "prt: small build n=%d: bounds+morton %.1f, sort %.1f, leaves %.1f, ploc %.1f (%u iterations), "
                   "collapse %.1f us; clusters after each iteration:", n, t(1) - t(0), t(2) - t(1), t(3) - t(2),
                   t(4) - t(3), w[7], t(5) - t(4));
      for (uint32_t k = 0; k < w[7] && k < 40; k++) std::fprintf(stderr, " %u", w[20 + k]);
      std::fprintf(stderr, "; ploc split: neighbours %.1f, merge %.1f, compaction %.1f us\n", w[60] / 100.0,
                   w[61] / 100.0, w[62] / 100.0);
    }
  }
  return hipGetLastError();
}

hipError_t launch_tlas_commit(hipStream_t s, const TlasMeta* mb, const Node8* nb, const uint32_t* sb,
                              const uint32_t* ob, TlasMeta* mf, Node8* nf, uint32_t* sf, uint32_t* of,
                              uint32_t* rejected) {
  hipLaunchKernelGGL(k_tlas_commit, dim3(1), dim3(kTlasSmallThreads), 0, s, mb, nb, sb, ob, mf, nf, sf, of, rejected);
  return hipGetLastError();
}

hipError_t launch_tlas_refit_meta(hipStream_t s, const InstDev* inst, const TlasMeta* meta, const uint32_t* order,
                                  Node8* nodes, const uint32_t* slot, float* aabb) {
  hipLaunchKernelGGL(k_tlas_refit_meta, dim3(1), dim3(kTlasSmallThreads), 0, s, inst, meta, order, nodes, slot, aabb);
  return hipGetLastError();
}

TlasMeta tlas_meta(const TlasTopo& T, uint32_t n_nodes) {
  TlasMeta m{};
  m.n_nodes = n_nodes;
  m.nlevels = (uint32_t)std::min<size_t>(T.level_cnt.size(), kTlasMaxLevels);
  m.depth = m.nlevels;
  m.valid = 1u;
  for (uint32_t l = 0; l < m.nlevels; l++) {
    m.level_off[l] = T.level_off[l];
    m.level_cnt[l] = T.level_cnt[l];
  }
  return m;
}

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
