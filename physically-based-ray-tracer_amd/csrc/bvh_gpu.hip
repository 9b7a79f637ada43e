// bvh_gpu.hip -- on-device BLAS build (the reference builds on the CPU,
// Core/tiny_bvh.h:1968-2284 BVH::Build / 3706-3781 BuildHQ, then BVH8_CPU's collapse).
//
// LBVH (Karras 2012, "Maximizing Parallelism in the Construction of BVHs, Octrees, and k-d Trees"):
//   1. centroid bounds (ordered-int atomics), 30-bit Morton code per triangle, key = code << 32 | index
//   2. hipcub radix sort of the 64-bit keys (unique keys: no duplicate-code special case)
//   3. binary radix tree: one thread per internal node finds its range and split from common prefixes
//   4. boxes bottom-up: one thread per leaf walks towards the root; the second child to arrive at a node
//      (agent atomic) unions both boxes.  Boxes are stored write-through (sc1) and read with sc1 loads
//      after the atomic, the in-launch hand-off of MI355X_MICROARCH.md (per-XCD L2s are not coherent)
//      In the same bottom-up pass, the SAH-optimal 8-wide collapse table of every internal node (Ylitie, Karras,
//      Laine 2017 sec. 3.1, as bvh_build.cpp WideDp): C(n, i) = cheapest cost of subtree n in at most i slots,
//      from its children's tables, in double, with the chosen split of the slots (Dk) and the leaf decision
//   5. 8-wide collapse, one launch per level: a wide node takes the <= 8 slots the table chose for it (a slot
//      whose single-slot form is a leaf becomes a leaf child with all its triangles, contiguous in key order).
//      Nodes are quantised and laid out exactly as the host builder's Node8 (bvh_build.h): interior
//      children contiguous (one atomic per node), leaf triangles contiguous (one atomic per node)
//   (LBVH and PLOC trees can be refined by treelet restructuring before step 5, PRT_TRBVH: see k_trbvh)
// The result is a different tree from the host's SAH build, so traversal cost differs; hits do not (the
// hit rule is BVH-independent), which is what the GPU tests check.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "bvh_build.h"
#include "bvh_gpu.h"

namespace prt {

namespace {

constexpr int kB = 256;
inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kB - 1) / kB); }

__device__ __forceinline__ uint32_t ord(float f) {  // float -> order-preserving uint
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every third bit
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<uint32_t*>(const_cast<float*>(p)), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1_d(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1_d(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<double*>(p)),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// collapse table of one internal node: C[1..8] (slot 0 unused), and in `dec` the decisions:
// bits 0-23: Dk[j] for j = 2..8 (3 bits each: the left child's share 1..7), bits 24-30: prev[i] for i = 2..8
// (C(n, i) == C(n, i - 1): use fewer slots), bit 31: leaf1 (the single-slot form of n is a leaf)
struct DpTab {
  double* C;      // 8 per internal node: C(n, i) at [8 n + i - 1]
  uint32_t* dec;  // 1 per internal node
};
constexpr double kDpNode = 1.0, kDpTri = 1.0;  // bvh_build.cpp kWideNodeCost / kWideTriCost
__device__ __forceinline__ double area6d(const float* b) {
  const double dx = (double)b[3] - b[0], dy = (double)b[4] - b[1], dz = (double)b[5] - b[2];
  return dx * dy + dy * dz + dz * dx;
}

// ---- 1. centroid bounds
__global__ void __launch_bounds__(kB) k_centroid_bounds(const float4* __restrict__ tri, uint32_t n, uint32_t* cb) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  float c[3] = {0.0f, 0.0f, 0.0f};
  const bool ok = i < n;
  if (ok) {
    const float4 a = tri[3 * i], b = tri[3 * i + 1], d = tri[3 * i + 2];
    c[0] = (a.x + b.x + d.x) * (1.0f / 3.0f);
    c[1] = (a.y + b.y + d.y) * (1.0f / 3.0f);
    c[2] = (a.z + b.z + d.z) * (1.0f / 3.0f);
  }
  for (int k = 0; k < 3; k++) {
    uint32_t lo = ok ? ord(c[k]) : 0xFFFFFFFFu, hi = ok ? ord(c[k]) : 0u;
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
      hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    if ((threadIdx.x & 63u) == 0) {
      atomicMin(cb + k, lo);
      atomicMax(cb + 3 + k, hi);
    }
  }
}

// ---- 2. Morton keys
__global__ void __launch_bounds__(kB) k_morton(const float4* __restrict__ tri, uint32_t n, const uint32_t* cb,
                                               unsigned long long* keys) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  const float4 a = tri[3 * i], b = tri[3 * i + 1], d = tri[3 * i + 2];
  const float c[3] = {(a.x + b.x + d.x) * (1.0f / 3.0f), (a.y + b.y + d.y) * (1.0f / 3.0f),
                      (a.z + b.z + d.z) * (1.0f / 3.0f)};
  uint32_t q[3];
  for (int k = 0; k < 3; k++) {
    const float lo = unord(cb[k]), hi = unord(cb[3 + k]);
    const float ext = hi - lo;
    const float t = ext > 0.0f ? (c[k] - lo) / ext : 0.0f;
    q[k] = (uint32_t)fminf(fmaxf(t * 1024.0f, 0.0f), 1023.0f);
  }
  const uint32_t code = (spread10(q[0]) << 2) | (spread10(q[1]) << 1) | spread10(q[2]);
  keys[i] = ((unsigned long long)code << 32) | i;
}

// ---- 3. binary radix tree.  Internal nodes 0 .. n-2, leaf i = node n-1+i.
__device__ __forceinline__ int delta(const unsigned long long* k, int n, int i, int j) {
  if (j < 0 || j >= n) return -1;
  return __clzll(k[i] ^ k[j]);
}
__global__ void __launch_bounds__(kB) k_radix_tree(const unsigned long long* __restrict__ keys, int n, int* left,
                                                   int* right, int* parent, uint32_t* first, uint32_t* count) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= n - 1) return;
  const int d = delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1) >= 0 ? 1 : -1;
  const int dmin = delta(keys, n, i, i - d);
  int lmax = 2;
  while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
  int l = 0;
  for (int t = lmax >> 1; t >= 1; t >>= 1)
    if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(keys, n, i, j);
  int s = 0;
  for (int t = (l + 1) >> 1;; t = (t + 1) >> 1) {
    if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    if (t == 1) break;
  }
  const int g = i + s * d + min(d, 0);
  const int lo = min(i, j), hi = max(i, j);
  const int lc = (lo == g) ? (n - 1 + g) : g;
  const int rc = (hi == g + 1) ? (n - 1 + g + 1) : (g + 1);
  left[i] = lc;
  right[i] = rc;
  parent[lc] = i;
  parent[rc] = i;
  first[i] = (uint32_t)lo;
  count[i] = (uint32_t)(hi - lo + 1);
}

// collapse table of internal node p from its children's (a binary leaf, id >= n - 1: one triangle, every C its
// leaf cost); children's tables were written earlier in this launch (sc1, after the arrival atomic) or by an
// earlier launch
__device__ __forceinline__ void dp_node(const DpTab& dp, int p, int lc, int rc, const float* pb, const float* lb,
                                        const float* rb, int cnt, int n, int max_leaf) {
  double cl[9], cr[9];
  const double al = area6d(lb) * kDpTri, ar = area6d(rb) * kDpTri;
  for (int i = 1; i <= 8; i++) {
    cl[i] = lc >= n - 1 ? al : ld_sc1_d(dp.C + 8 * (size_t)lc + i - 1);
    cr[i] = rc >= n - 1 ? ar : ld_sc1_d(dp.C + 8 * (size_t)rc + i - 1);
  }
  const double A = fmax(area6d(pb), 1e-30);
  const double leafc = cnt <= max_leaf ? A * kDpTri * (double)cnt : 1e300;
  double D[9];
  uint32_t dec = 0;
  for (int j = 2; j <= 8; j++) {
    D[j] = 1e300;
    uint32_t bk = 1;
    for (int k = 1; k < j; k++) {
      const double c = cl[k] + cr[j - k];
      if (c < D[j]) { D[j] = c; bk = (uint32_t)k; }
    }
    dec |= bk << (3 * (j - 2));
  }
  const double intc = A * kDpNode + D[8];
  if (cnt <= max_leaf && leafc <= intc) dec |= 1u << 31;
  double C = fmin(leafc, intc);
  auto put = [&](size_t at, double v) { st_sc1_d(dp.C + at, v); };
  put(8 * (size_t)p, C);
  for (int i = 2; i <= 8; i++) {
    if (C <= D[i]) dec |= 1u << (24 + i - 2);
    else C = D[i];
    put(8 * (size_t)p + i - 1, C);
  }
  dp.dec[p] = dec;
}

// ---- 4. boxes bottom-up (flag[] zeroed before the launch)
__global__ void __launch_bounds__(kB) k_boxes(const float4* __restrict__ tri, const unsigned long long* __restrict__ keys,
                                              int n, const int* __restrict__ left, const int* __restrict__ right,
                                              const int* __restrict__ parent, float* box, uint32_t* flag,
                                              uint32_t* first, uint32_t* count, DpTab dp, int max_leaf) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= n) return;
  const uint32_t prim = (uint32_t)keys[i];
  const float4 a = tri[3 * prim], b = tri[3 * prim + 1], c = tri[3 * prim + 2];
  int node = n - 1 + i;
  float* bx = box + 6 * (size_t)node;
  st_sc1(bx + 0, fminf(fminf(a.x, b.x), c.x));
  st_sc1(bx + 1, fminf(fminf(a.y, b.y), c.y));
  st_sc1(bx + 2, fminf(fminf(a.z, b.z), c.z));
  st_sc1(bx + 3, fmaxf(fmaxf(a.x, b.x), c.x));
  st_sc1(bx + 4, fmaxf(fmaxf(a.y, b.y), c.y));
  st_sc1(bx + 5, fmaxf(fmaxf(a.z, b.z), c.z));
  first[node] = (uint32_t)i;
  count[node] = 1u;
  if (n == 1) return;
  while (node != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this node's box is out before the arrival
    const int p = parent[node];
    if (p < 0 || p >= n - 1) return;                    // malformed tree: the host checks the node count
    if (atomicAdd(flag + p, 1u) == 0u) return;          // the sibling's thread finishes the parent
    const int lc = left[p], rc = right[p];
    const float* l = box + 6 * (size_t)lc;
    const float* r = box + 6 * (size_t)rc;
    float* o = box + 6 * (size_t)p;
    float pb[6], lb[6], rb[6];
    for (int k = 0; k < 6; k++) { lb[k] = ld_sc1(l + k); rb[k] = ld_sc1(r + k); }
    for (int k = 0; k < 3; k++) { pb[k] = fminf(lb[k], rb[k]); st_sc1(o + k, pb[k]); }
    for (int k = 3; k < 6; k++) { pb[k] = fmaxf(lb[k], rb[k]); st_sc1(o + k, pb[k]); }
    if (dp.C) dp_node(dp, p, lc, rc, pb, lb, rb, (int)count[p], n, max_leaf);
    node = p;
  }
}

// ---- PLOC (Meister, Bittner 2018, "Parallel Locally-Ordered Clustering for Bounding Volume Hierarchy
// Construction"): clusters start as the Morton-ordered triangles; every iteration each cluster finds the
// neighbour within kPlocR places (in the current cluster order) whose merged box has the smallest surface area,
// mutual nearest neighbours merge into a new internal node, and the survivors are compacted in order.  Ties are
// broken by the pair's indices, so the globally best pair is always mutual and every iteration merges.
// Internal nodes take ids n-2, n-3, ... as they are created, so the root (created last) is node 0 and the
// LBVH node numbering (leaves n-1+i) and the collapse below apply unchanged; the collapse table of a node is
// filled when it is created, from its children's (created in earlier launches).
// search radius: 64 places (C4 rate on the resulting tree 3,327 / 3,428 / 3,534 / 3,492 / 3,466 Mrays/s at radius
// 16 / 32 / 64 / 128 / 256, build 51-59 ms throughout; scripts/gpu_ploc_ab.sh)
#ifndef PRT_PLOC_R
#define PRT_PLOC_R 64
#endif
constexpr int kPlocDefaultR = PRT_PLOC_R;

__global__ void __launch_bounds__(kB) k_ploc_leaves(const float4* __restrict__ tri,
                                                    const unsigned long long* __restrict__ keys, int n, float* box,
                                                    uint32_t* count, int* clus) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= n) return;
  const uint32_t prim = (uint32_t)keys[i];
  const float4 a = tri[3 * prim], b = tri[3 * prim + 1], c = tri[3 * prim + 2];
  float* bx = box + 6 * (size_t)(n - 1 + i);
  bx[0] = fminf(fminf(a.x, b.x), c.x); bx[1] = fminf(fminf(a.y, b.y), c.y); bx[2] = fminf(fminf(a.z, b.z), c.z);
  bx[3] = fmaxf(fmaxf(a.x, b.x), c.x); bx[4] = fmaxf(fmaxf(a.y, b.y), c.y); bx[5] = fmaxf(fmaxf(a.z, b.z), c.z);
  count[n - 1 + i] = 1u;
  clus[i] = n - 1 + i;
}

// nearest neighbour of every cluster (by merged surface area) within kPlocR places; the block's boxes (plus the
// kPlocR on either side) staged in LDS
template <int kPlocR>
__global__ void __launch_bounds__(kB) k_ploc_nn(const int* __restrict__ clus, int m, const float* __restrict__ box,
                                                int* nn) {
  __shared__ float sb[6 * (kB + 2 * kPlocR)];
  const int b0 = (int)(blockIdx.x * kB) - kPlocR;
  for (int t = threadIdx.x; t < kB + 2 * kPlocR; t += kB) {
    const int j = b0 + t;
    if (j >= 0 && j < m) {
      const float* bx = box + 6 * (size_t)clus[j];
      for (int k = 0; k < 6; k++) sb[6 * t + k] = bx[k];
    }
  }
  __syncthreads();
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= m) return;
  const float* bi = sb + 6 * (i - b0);
  float best = 3.4e38f;
  int bj = -1;
  for (int j = max(0, i - kPlocR); j <= min(m - 1, i + kPlocR); j++) {
    if (j == i) continue;
    const float* bj6 = sb + 6 * (j - b0);
    const float dx = fmaxf(bi[3], bj6[3]) - fminf(bi[0], bj6[0]);
    const float dy = fmaxf(bi[4], bj6[4]) - fminf(bi[1], bj6[1]);
    const float dz = fmaxf(bi[5], bj6[5]) - fminf(bi[2], bj6[2]);
    const float a = dx * dy + dy * dz + dz * dx;
    // ties: the pair (min index, max index) that sorts first, the same order from both ends of a pair
    const bool better = a < best || (a == best && bj >= 0 && (min(i, j) < min(i, bj) ||
                                                              (min(i, j) == min(i, bj) && max(i, j) < max(i, bj))));
    if (bj < 0 || better) { best = a; bj = j; }
  }
  nn[i] = bj;
}

// mutual nearest neighbours merge (the lower index creates the node and keeps the slot); ctr[0] counts down the
// internal node ids
__global__ void __launch_bounds__(kB) k_ploc_merge(const int* __restrict__ clus, int m, const int* __restrict__ nn,
                                                   float* box, int* left, int* right, uint32_t* count, int* out,
                                                   int* keep, uint32_t* ctr, DpTab dp, int n, int max_leaf) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= m) return;
  const int j = nn[i];
  const bool mutual = j >= 0 && nn[j] == i;
  if (mutual && i > j) {  // merged into the cluster at j
    keep[i] = 0;
    return;
  }
  keep[i] = 1;
  if (!mutual) {
    out[i] = clus[i];
    return;
  }
  const int lc = clus[i], rc = clus[j];
  const int p = (int)atomicSub(ctr, 1u) - 1;
  if (p < 0) { atomicOr(ctr + 3, 0x80000000u); out[i] = lc; return; }
  float lb[6], rb[6], pb[6];
  for (int k = 0; k < 6; k++) { lb[k] = box[6 * (size_t)lc + k]; rb[k] = box[6 * (size_t)rc + k]; }
  for (int k = 0; k < 3; k++) { pb[k] = fminf(lb[k], rb[k]); pb[3 + k] = fmaxf(lb[3 + k], rb[3 + k]); }
  for (int k = 0; k < 6; k++) box[6 * (size_t)p + k] = pb[k];
  left[p] = lc;
  right[p] = rc;
  count[p] = count[lc] + count[rc];
  if (dp.C) dp_node(dp, p, lc, rc, pb, lb, rb, (int)count[p], n, max_leaf);
  out[i] = p;
}

// ---- 5. box helpers of the collapse (bvh_build.cpp's inflation and grid exponent)
__device__ __forceinline__ void inflate(float* lo, float* hi) {  // inflate_box (bvh_build.cpp)
  for (int k = 0; k < 3; k++) {
    const float ext = fmaxf(fabsf(lo[k]), fabsf(hi[k]));
    const float pad = ext * 1e-6f + 1e-7f;
    lo[k] -= pad;
    hi[k] += pad;
  }
}
__device__ __forceinline__ uint8_t grid_exp(double ext, double qmax) {  // grid_exponent (bvh_build.cpp)
  if (!(ext > 0)) return 1;
  int e = (int)ceil(log2(ext / qmax));
  while (ldexp(qmax, e) < ext) e++;
  while (e > -126 && ldexp(qmax, e - 1) >= ext) e--;
  return (uint8_t)min(254, max(1, e + 127));
}

// ---- treelet restructuring of the binary tree before the collapse (Karras, Aila 2013, "Fast Parallel
// Construction of High-Quality Bounding Volume Hierarchies"), PRT_TRBVH passes (0 = off): one thread per leaf
// walks towards the root; the second child to arrive at a node (agent atomic, as k_boxes) forms the treelet of up
// to kTreeletLeaves subtrees below it (opening the largest-area treelet leaf until full), finds the binary
// topology over them with the least SAH cost by dynamic programming over the subsets, and rewires the treelet's
// internal nodes when that is cheaper.  Subtrees below a node are final when it is processed, nodes above it
// untouched, so treelets of different threads never overlap.  Boxes, counts, costs and links move between threads
// with sc1 loads / stores after the arrival atomic (per-XCD L2s, MI355X_MICROARCH.md).  The restructured tree's
// subtrees are no longer Morton key ranges: the collapse walks them, and the collapse table is rebuilt.
constexpr int kTreeletLeaves = 7;
constexpr float kTrNode = 1.0f, kTrTri = 1.0f;  // binary SAH weights, as kDpNode / kDpTri

__device__ __forceinline__ int ld_sc1_i(const int* p) {
  return (int)__hip_atomic_load(reinterpret_cast<uint32_t*>(const_cast<int*>(p)), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_i(int* p, int v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float area_of(const float* lo, const float* hi) {
  const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
  return dx * dy + dy * dz + dz * dx;
}

// parent links of a tree given by left / right (PLOC builds none)
__global__ void __launch_bounds__(kB) k_parents(const int* __restrict__ left, const int* __restrict__ right, int n,
                                                int* parent) {
  const int p = (int)(blockIdx.x * kB + threadIdx.x);
  if (p == 0) parent[0] = -1;
  if (p >= n - 1) return;
  const int nn = 2 * n - 1, l = left[p], r = right[p];
  if (l > 0 && l < nn) parent[l] = p;
  if (r > 0 && r < nn) parent[r] = p;
}

__global__ void __launch_bounds__(kB) k_trbvh(int n, int* left, int* right, int* parent, float* box, uint32_t* count,
                                              float* cost, uint32_t* flag, uint32_t* err) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= n) return;
  const int nn = 2 * n - 1;
  int node = n - 1 + i;
  {
    const float* b = box + 6 * (size_t)node;
    float lo[3], hi[3];
    for (int k = 0; k < 3; k++) { lo[k] = ld_sc1(b + k); hi[k] = ld_sc1(b + 3 + k); }
    st_sc1(cost + node, kTrTri * area_of(lo, hi));
  }
  while (node != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this subtree's records are out before the arrival
    const int p = ld_sc1_i(parent + node);
    if (p < 0 || p >= n - 1) { atomicOr(err, 1u); return; }
    if (atomicAdd(flag + p, 1u) == 0u) return;  // the sibling's thread finishes p
    node = p;
    // the treelet below p: internal nodes I (p first), leaves L (subtree roots)
    int L[kTreeletLeaves], I[kTreeletLeaves - 1];
    float lbx[kTreeletLeaves][6];
    int nl = 0, ni = 0;
    I[ni++] = p;
    L[nl++] = ld_sc1_i(left + p);
    L[nl++] = ld_sc1_i(right + p);
    bool bad = false;
    for (int j = 0; j < 2; j++) bad |= L[j] < 0 || L[j] >= nn;
    if (bad) { atomicOr(err, 2u); return; }
    for (int j = 0; j < 2; j++)
      for (int k = 0; k < 6; k++) lbx[j][k] = ld_sc1(box + 6 * (size_t)L[j] + k);
    while (nl < kTreeletLeaves) {  // open the largest-area interior treelet leaf
      int bj = -1;
      float ba = -1.0f;
      for (int j = 0; j < nl; j++)
        if (L[j] < n - 1) {
          const float a = area_of(lbx[j], lbx[j] + 3);
          if (a > ba) { ba = a; bj = j; }
        }
      if (bj < 0) break;
      const int v = L[bj];
      const int lv = ld_sc1_i(left + v), rv = ld_sc1_i(right + v);
      if (lv < 0 || lv >= nn || rv < 0 || rv >= nn) { atomicOr(err, 4u); return; }
      I[ni++] = v;
      L[bj] = lv;
      L[nl] = rv;
      for (int k = 0; k < 6; k++) { lbx[bj][k] = ld_sc1(box + 6 * (size_t)lv + k); lbx[nl][k] = ld_sc1(box + 6 * (size_t)rv + k); }
      nl++;
    }
    float lcost[kTreeletLeaves];
    for (int j = 0; j < nl; j++) lcost[j] = ld_sc1(cost + L[j]);
    float pb[6];
    for (int k = 0; k < 3; k++) { pb[k] = 3.4e38f; pb[3 + k] = -3.4e38f; }
    for (int j = 0; j < nl; j++)
      for (int k = 0; k < 3; k++) { pb[k] = fminf(pb[k], lbx[j][k]); pb[3 + k] = fmaxf(pb[3 + k], lbx[j][3 + k]); }
    // current cost of the treelet: rebuilt bottom-up over its internal nodes (I is in pre-order: reverse it)
    const int full = (1 << nl) - 1;
    float ca[1 << kTreeletLeaves], cs[1 << kTreeletLeaves];
    uint8_t part[1 << kTreeletLeaves];
    for (int S = 1; S <= full; S++) {
      float lo[3] = {3.4e38f, 3.4e38f, 3.4e38f}, hi[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
      for (int j = 0; j < nl; j++)
        if ((S >> j) & 1)
          for (int k = 0; k < 3; k++) { lo[k] = fminf(lo[k], lbx[j][k]); hi[k] = fmaxf(hi[k], lbx[j][3 + k]); }
      ca[S] = area_of(lo, hi);
    }
    for (int S = 1; S <= full; S++) {  // subsets of S are numerically smaller: already solved
      if ((S & (S - 1)) == 0) {
        cs[S] = lcost[__builtin_ctz(S)];
        part[S] = 0;
        continue;
      }
      const int low = S & -S;
      float best = 3.4e38f;
      int bp = low;
      for (int P = (S - 1) & S; P; P = (P - 1) & S)
        if (P & low) {
          const float c = cs[P] + cs[S ^ P];
          if (c < best) { best = c; bp = P; }
        }
      cs[S] = kTrNode * ca[S] + best;
      part[S] = (uint8_t)bp;
    }
    const float old = kTrNode * area_of(pb, pb + 3) + ld_sc1(cost + ld_sc1_i(left + p)) + ld_sc1(cost + ld_sc1_i(right + p));
    if (nl >= 3 && cs[full] < old * 0.9999f) {
      // rewire: pre-order over the chosen partitions, internal nodes taken from I in order
      int stS[kTreeletLeaves], stN[kTreeletLeaves], sp = 0, used = 1;
      int oN[kTreeletLeaves - 1], oL[kTreeletLeaves - 1], oR[kTreeletLeaves - 1], no = 0;
      stS[sp] = full; stN[sp++] = p;
      while (sp > 0 && !bad) {
        const int S = stS[--sp], id = stN[sp];
        const int P = part[S], Q = S ^ P;
        int ch[2];
        const int sub[2] = {P, Q};
        for (int h = 0; h < 2; h++) {
          const int X = sub[h];
          if ((X & (X - 1)) == 0) {
            ch[h] = L[__builtin_ctz(X)];
          } else {
            if (used >= ni || sp >= kTreeletLeaves) { bad = true; break; }
            ch[h] = I[used++];
            stS[sp] = X; stN[sp++] = ch[h];
          }
        }
        if (bad || no >= kTreeletLeaves - 1) { bad = true; break; }
        oN[no] = id; oL[no] = ch[0]; oR[no] = ch[1]; no++;
      }
      if (bad || used != ni) { atomicOr(err, 8u); return; }
      // links, then boxes / counts / costs children first (reverse pre-order)
      for (int j = 0; j < no; j++) {
        st_sc1_i(left + oN[j], oL[j]);
        st_sc1_i(right + oN[j], oR[j]);
        st_sc1_i(parent + oL[j], oN[j]);
        st_sc1_i(parent + oR[j], oN[j]);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int j = no - 1; j >= 0; j--) {
        const int id = oN[j], l = oL[j], r = oR[j];
        float lo[3], hi[3];
        for (int k = 0; k < 3; k++) {
          lo[k] = fminf(ld_sc1(box + 6 * (size_t)l + k), ld_sc1(box + 6 * (size_t)r + k));
          hi[k] = fmaxf(ld_sc1(box + 6 * (size_t)l + 3 + k), ld_sc1(box + 6 * (size_t)r + 3 + k));
        }
        for (int k = 0; k < 3; k++) { st_sc1(box + 6 * (size_t)id + k, lo[k]); st_sc1(box + 6 * (size_t)id + 3 + k, hi[k]); }
        st_sc1_u(count + id, ld_sc1_u(count + l) + ld_sc1_u(count + r));
        st_sc1(cost + id, kTrNode * area_of(lo, hi) + ld_sc1(cost + l) + ld_sc1(cost + r));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // read back by the next (parent) record
      }
    } else {
      st_sc1(cost + p, old);
    }
  }
}

// the collapse table over the restructured tree (boxes final): the dp_node pass of k_boxes, bottom-up
__global__ void __launch_bounds__(kB) k_dp_rebuild(int n, const int* __restrict__ left, const int* __restrict__ right,
                                                   const int* __restrict__ parent, const float* __restrict__ box,
                                                   const uint32_t* __restrict__ count, uint32_t* flag, DpTab dp,
                                                   int max_leaf, uint32_t* err) {
  const int i = (int)(blockIdx.x * kB + threadIdx.x);
  if (i >= n) return;
  int node = n - 1 + i;
  while (node != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int p = parent[node];
    if (p < 0 || p >= n - 1) { atomicOr(err, 16u); return; }
    if (atomicAdd(flag + p, 1u) == 0u) return;
    const int lc = left[p], rc = right[p];
    float pb[6], lb[6], rb[6];
    for (int k = 0; k < 6; k++) { lb[k] = box[6 * (size_t)lc + k]; rb[k] = box[6 * (size_t)rc + k]; pb[k] = box[6 * (size_t)p + k]; }
    dp_node(dp, p, lc, rc, pb, lb, rb, (int)count[p], n, max_leaf);
    node = p;
  }
}

struct Task {
  int n2;       // binary node
  uint32_t n8;  // wide node slot
};

// one wide node of the collapse: task tk (binary node -> wide node slot); the next level's tasks go to next
__device__ __forceinline__ void collapse_task(const Task tk, const float4* __restrict__ tri,
                                              const unsigned long long* __restrict__ keys, int n,
                                              const int* __restrict__ left, const int* __restrict__ right,
                                              const float* __restrict__ box, const uint32_t* __restrict__ first,
                                              const uint32_t* __restrict__ count, int max_leaf, Task* next,
                                              uint32_t* ctr, Node8* nodes, TriMT* tris, const DpTab& dp) {
  const int nn = 2 * n - 1;
  if (tk.n2 < 0 || tk.n2 >= nn || tk.n8 >= (uint32_t)n) { atomicOr(ctr + 3, 0x80000000u); return; }
  // a child slot's form: leaf (all its triangles) or a wide node of its own
  auto is_leaf = [&](int v) { return v >= n - 1 || (dp.dec[v] >> 31) != 0; };  // (n == 1: no table, one leaf)
  int ch[8];
  int nc = 0;
  if (!is_leaf(tk.n2)) {
    // the slots the table chose: expand(n) = collect(left, Dk[n][8]) + collect(right, 8 - Dk[n][8]), where
    // collect(v, i) = v if i == 1 or v is a leaf / its own form; collect(v, i - 1) if prev; else split again
    int st_n[16], st_i[16], sp = 0;
    const uint32_t d0 = dp.dec[tk.n2];
    const int k0 = (int)((d0 >> 18) & 7u);  // Dk[n][8]
    st_n[sp] = right[tk.n2]; st_i[sp++] = 8 - k0;
    st_n[sp] = left[tk.n2]; st_i[sp++] = k0;
    while (sp > 0 && nc < 8) {
      const int v = st_n[--sp];
      int i = st_i[sp];
      if (v >= n - 1 || i <= 1) { ch[nc++] = v; continue; }
      const uint32_t d = dp.dec[v];
      while (i > 1 && ((d >> (24 + i - 2)) & 1u)) i--;
      if (i <= 1) { ch[nc++] = v; continue; }
      const int k = (int)((d >> (3 * (i - 2))) & 7u);
      if (sp + 2 > 16) { atomicOr(ctr + 3, 0x80000000u); return; }
      st_n[sp] = right[v]; st_i[sp++] = i - k;
      st_n[sp] = left[v]; st_i[sp++] = k;
    }
  } else {
    ch[nc++] = tk.n2;
  }
  for (int i = 0; i < nc; i++)
    if (ch[i] < 0 || ch[i] >= nn) { atomicOr(ctr + 3, 0x80000000u); return; }
  float clo[8][3], chi[8][3];
  double nlo[3] = {1e300, 1e300, 1e300}, nhi[3] = {-1e300, -1e300, -1e300};
  for (int i = 0; i < nc; i++) {
    const float* b = box + 6 * (size_t)ch[i];
    for (int k = 0; k < 3; k++) { clo[i][k] = b[k]; chi[i][k] = b[3 + k]; }
    inflate(clo[i], chi[i]);
    for (int k = 0; k < 3; k++) {
      nlo[k] = fmin(nlo[k], (double)clo[i][k]);
      nhi[k] = fmax(nhi[k], (double)chi[i][k]);
    }
  }
  // octant slots: slot s holds the child that comes first for rays of octant s (greedy assignment)
  int child_in[8];
  for (int s = 0; s < 8; s++) child_in[s] = -1;
  {
    double pc[3];
    for (int k = 0; k < 3; k++) pc[k] = 0.5 * (nlo[k] + nhi[k]);
    // each child's centroid offset once (the greedy rounds below re-read it; the same double operations, so the
    // same costs bit for bit as computing it per pair)
    // (loops unrolled over all 8 children: constant indices keep cc in registers)
    double cc[8][3];
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int k = 0; k < 3; k++) cc[i][k] = i < nc ? 0.5 * ((double)clo[i][k] + (double)chi[i][k]) - pc[k] : 0.0;
    uint32_t used_c = 0, used_s = 0;
    for (int m = 0; m < nc; m++) {
      double best = 1e300;
      int bi = -1, bs = -1;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (i >= nc || (used_c & (1u << i))) continue;
#pragma unroll
        for (int s = 0; s < 8; s++) {
          if (used_s & (1u << s)) continue;
          double d = 0;
#pragma unroll
          for (int k = 0; k < 3; k++) d += ((s >> k) & 1) ? -cc[i][k] : cc[i][k];
          if (d < best) { best = d; bi = i; bs = s; }
        }
      }
      used_c |= 1u << bi;
      used_s |= 1u << bs;
      child_in[bs] = bi;
    }
  }
  Node8 nd;
  uint8_t* raw = reinterpret_cast<uint8_t*>(&nd);
  for (int b = 0; b < (int)sizeof(Node8); b++) raw[b] = 0;
  nd.px = (float)nlo[0]; nd.py = (float)nlo[1]; nd.pz = (float)nlo[2];
  const double p[3] = {(double)nd.px, (double)nd.py, (double)nd.pz};
  uint8_t e[3];
  for (int k = 0; k < 3; k++) e[k] = grid_exp(nhi[k] - p[k], 255.0);
  nd.ex = e[0]; nd.ey = e[1]; nd.ez = e[2];
  // the grid step 2^(e - 127) and its exact inverse: (x - p) * 2^(127 - e) is the quotient (x - p) / 2^(e - 127) bit
  // for bit, without a double division
  const double isc[3] = {ldexp(1.0, 127 - (int)e[0]), ldexp(1.0, 127 - (int)e[1]), ldexp(1.0, 127 - (int)e[2])};
  uint32_t ninterior = 0, ntri = 0;
  for (int i = 0; i < nc; i++) {
    if (is_leaf(ch[i])) ntri += count[ch[i]];
    else ninterior++;
  }
  if ((uint32_t)nc > ninterior) atomicAdd(ctr + 3, (uint32_t)nc - ninterior);  // leaf children
  nd.child_base = ninterior ? atomicAdd(ctr + 0, ninterior) : 0u;
  nd.tri_base = ntri ? atomicAdd(ctr + 1, ntri) : 0u;
  const uint32_t tbase = ninterior ? atomicAdd(ctr + 2, ninterior) : 0u;  // next-level task slots
  if (nd.child_base + ninterior > (uint32_t)n || nd.tri_base + ntri > (uint32_t)n || tbase + ninterior > (uint32_t)n) {
    atomicOr(ctr + 3, 0x80000000u);  // capacity exceeded: cannot happen for a well-formed radix tree
    return;
  }
  uint32_t nextchild = nd.child_base, tri_off = 0, tslot = tbase;
  for (int s = 0; s < 8; s++) {
    const int i = child_in[s];
    if (i < 0) {
      nd.qlox[s] = nd.qloy[s] = nd.qloz[s] = 255;
      nd.qhix[s] = nd.qhiy[s] = nd.qhiz[s] = 0;
      continue;
    }
    uint8_t* ql[3] = {&nd.qlox[s], &nd.qloy[s], &nd.qloz[s]};
    uint8_t* qh[3] = {&nd.qhix[s], &nd.qhiy[s], &nd.qhiz[s]};
    for (int k = 0; k < 3; k++) {
      *ql[k] = (uint8_t)fmin(255.0, fmax(0.0, floor(((double)clo[i][k] - p[k]) * isc[k])));
      *qh[k] = (uint8_t)fmin(255.0, fmax(0.0, ceil(((double)chi[i][k] - p[k]) * isc[k])));
    }
    const int c = ch[i];
    if (is_leaf(c)) {
      // the leaf child's triangles: a key range (LBVH subtrees are contiguous in Morton order), or (PLOC,
      // first == nullptr) the binary leaves under c, at most max_leaf of them
      uint32_t kidx[8];
      uint32_t cnt = 0;
      if (c >= n - 1) {
        kidx[cnt++] = (uint32_t)(c - (n - 1));
      } else if (first) {
        cnt = min(count[c], 8u);
        for (uint32_t j = 0; j < cnt; j++) kidx[j] = first[c] + j;
      } else {
        int st[8], sp = 0;
        st[sp++] = c;
        while (sp > 0 && cnt < 8) {
          const int v = st[--sp];
          if (v >= n - 1) { kidx[cnt++] = (uint32_t)(v - (n - 1)); continue; }
          if (sp + 2 > 8) break;
          st[sp++] = right[v];
          st[sp++] = left[v];
        }
      }
      if (cnt != count[c] || cnt > 7) { atomicOr(ctr + 3, 0x80000000u); return; }
      for (uint32_t j = 0; j < cnt; j++) {
        const uint32_t pr = (uint32_t)keys[kidx[j]];
        const float4 a = tri[3 * pr], b = tri[3 * pr + 1], d = tri[3 * pr + 2];
        TriMT m;
        m.v0[0] = a.x; m.v0[1] = a.y; m.v0[2] = a.z;
        m.e1[0] = b.x - a.x; m.e1[1] = b.y - a.y; m.e1[2] = b.z - a.z;  // e1 = v1 - v0 (tiny_bvh.h:4614-4616)
        m.e2[0] = d.x - a.x; m.e2[1] = d.y - a.y; m.e2[2] = d.z - a.z;
        m.prim = pr; m.pad1 = 0.0f; m.pad2 = 0.0f;
        tris[nd.tri_base + tri_off + j] = m;
      }
      nd.meta[s] = (uint8_t)((tri_off << 3) | cnt);
      tri_off += cnt;
    } else {
      nd.imask |= (uint8_t)(1u << s);
      next[tslot++] = Task{c, nextchild++};
    }
  }
  nodes[tk.n8] = nd;
}

__global__ void __launch_bounds__(kB) k_collapse(const float4* __restrict__ tri, const unsigned long long* __restrict__ keys,
                                                 int n, const int* __restrict__ left, const int* __restrict__ right,
                                                 const float* __restrict__ box, const uint32_t* __restrict__ first,
                                                 const uint32_t* __restrict__ count, int max_leaf,
                                                 const Task* __restrict__ tasks, uint32_t ntasks, Task* next,
                                                 uint32_t* ctr, Node8* nodes, TriMT* tris, DpTab dp) {
  const uint32_t t = blockIdx.x * kB + threadIdx.x;
  if (t >= ntasks) return;
  collapse_task(tasks[t], tri, keys, n, left, right, box, first, count, max_leaf, next, ctr, nodes, tris, dp);
}

// ShadeTri.pad[0] = the primitive's TriMT record (the cooperative traversal tail, prt_persist.h)
__global__ void __launch_bounds__(kB) k_prim_records(const TriMT* __restrict__ tris, uint32_t n, uint32_t tri_base,
                                                     ShadeTri* stri, uint32_t prim_base) {
  const uint32_t g = blockIdx.x * kB + threadIdx.x;
  if (g >= n) return;
  stri[prim_base + tris[g].prim].pad[0] = tri_base + g;
}

// rebase one mesh's nodes into the concatenated arrays
__global__ void __launch_bounds__(kB) k_rebase(Node8* nodes, uint32_t n, uint32_t node_base, uint32_t tri_base) {
  const uint32_t i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  nodes[i].child_base += node_base;
  nodes[i].tri_base += tri_base;
}

}  // namespace

// the build's scratch is stream-ordered (hipMallocAsync / hipFreeAsync on the build stream): no device-wide
// synchronisation, so a build on a side stream (the instance BVH's rebuild, prt_api.cpp) overlaps queued frames
inline void afree(void* p, hipStream_t s) {
  if (p) (void)hipFreeAsync(p, s);
}

#define GB_TRY(x)                          \
  do {                                     \
    const hipError_t e_ = (x);             \
    if (e_ != hipSuccess) return e_;       \
  } while (0)

hipError_t gpu_build_blas8(hipStream_t s, const float* tri_dev, int32_t n_tris, int max_leaf, Node8* nodes_out,
                           TriMT* tris_out, GpuBlasInfo* info, bool ploc, std::vector<uint32_t>* level_ends,
                           int trbvh, int ploc_radius) {
  const int n = n_tris;
  if (n <= 0) return hipErrorInvalidValue;
  const size_t nn = 2 * (size_t)n - 1;
  // scratch: keys x2, left/right/parent/first/count/flag, boxes, two task arrays, counters
  unsigned long long *keys = nullptr, *keys2 = nullptr;
  int *left = nullptr, *right = nullptr, *parent = nullptr;
  uint32_t *first = nullptr, *count = nullptr, *flag = nullptr, *ctr = nullptr, *cb = nullptr;
  float* box = nullptr;
  DpTab dp{nullptr, nullptr};
  Task *ta = nullptr, *tb = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  hipError_t err = hipSuccess;
  auto fail = [&](hipError_t e) {
    afree(keys, s); afree(keys2, s); afree(left, s); afree(right, s); afree(parent, s);
    afree(first, s); afree(count, s); afree(flag, s); afree(ctr, s); afree(cb, s);
    afree(box, s); afree(ta, s); afree(tb, s); afree(tmp, s);
    afree(dp.C, s); afree(dp.dec, s);
    return e;
  };
  const float4* tri = reinterpret_cast<const float4*>(tri_dev);
  if ((err = hipMallocAsync(reinterpret_cast<void**>(&keys), 8 * (size_t)n, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&keys2), 8 * (size_t)n, s)) ||
      (err = hipMallocAsync(reinterpret_cast<void**>(&left), 4 * nn, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&right), 4 * nn, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&parent), 4 * nn, s)) ||
      (err = hipMallocAsync(reinterpret_cast<void**>(&first), 4 * nn, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&count), 4 * nn, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&flag), 4 * nn, s)) ||
      (err = hipMallocAsync(reinterpret_cast<void**>(&box), 24 * nn, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&ta), sizeof(Task) * (size_t)n, s)) ||
      (err = hipMallocAsync(reinterpret_cast<void**>(&tb), sizeof(Task) * (size_t)n, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&ctr), 16, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&cb), 24, s)))
    return fail(err);
  if (n > 1) {
    if ((err = hipMallocAsync(reinterpret_cast<void**>(&dp.C), 8 * sizeof(double) * (size_t)(n - 1), s)) ||
        (err = hipMallocAsync(reinterpret_cast<void**>(&dp.dec), sizeof(uint32_t) * (size_t)(n - 1), s)))
      return fail(err);
  }
  const uint32_t init_cb[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
  if ((err = hipMemcpyAsync(cb, init_cb, 24, hipMemcpyHostToDevice, s))) return fail(err);
  hipLaunchKernelGGL(k_centroid_bounds, dim3(grid_of(n)), dim3(kB), 0, s, tri, (uint32_t)n, cb);
  hipLaunchKernelGGL(k_morton, dim3(grid_of(n)), dim3(kB), 0, s, tri, (uint32_t)n, cb, keys);
  if ((err = hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, keys, keys2, n, 0, 64, s))) return fail(err);
  if ((err = hipMallocAsync(reinterpret_cast<void**>(&tmp), tmp_bytes, s))) return fail(err);
  if ((err = hipcub::DeviceRadixSort::SortKeys(tmp, tmp_bytes, keys, keys2, n, 0, 64, s))) return fail(err);
  if (ploc) {
    // clusters: the Morton-ordered leaves; iterate nearest-neighbour / merge / compact down to the root
    int *clus = nullptr, *clus2 = nullptr, *nnb = nullptr, *keep = nullptr, *nsel = nullptr;
    void* stmp = nullptr;
    size_t stmp_bytes = 0;
    auto pfree = [&]() {
      afree(clus, s); afree(clus2, s); afree(nnb, s); afree(keep, s); afree(nsel, s);
      afree(stmp, s);
    };
    if ((err = hipMallocAsync(reinterpret_cast<void**>(&clus), 4 * (size_t)n, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&clus2), 4 * (size_t)n, s)) ||
        (err = hipMallocAsync(reinterpret_cast<void**>(&nnb), 4 * (size_t)n, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&keep), 4 * (size_t)n, s)) ||
        (err = hipMallocAsync(reinterpret_cast<void**>(&nsel), 4, s)) ||
        (err = hipcub::DeviceSelect::Flagged(nullptr, stmp_bytes, clus2, keep, clus, nsel, n, s)) ||
        (err = hipMallocAsync(reinterpret_cast<void**>(&stmp), stmp_bytes, s))) {
      pfree();
      return fail(err);
    }
    const uint32_t c0p[4] = {(uint32_t)(n - 1), 0u, 0u, 0u};
    if ((err = hipMemcpyAsync(ctr, c0p, 16, hipMemcpyHostToDevice, s))) { pfree(); return fail(err); }
    hipLaunchKernelGGL(k_ploc_leaves, dim3(grid_of(n)), dim3(kB), 0, s, tri, keys2, n, box, count, clus);
    int m = n;
    while (m > 1 && !err) {
      if (ploc_radius >= 512) hipLaunchKernelGGL(k_ploc_nn<512>, dim3(grid_of(m)), dim3(kB), 0, s, clus, m, box, nnb);
      else hipLaunchKernelGGL(k_ploc_nn<kPlocDefaultR>, dim3(grid_of(m)), dim3(kB), 0, s, clus, m, box, nnb);
      hipLaunchKernelGGL(k_ploc_merge, dim3(grid_of(m)), dim3(kB), 0, s, clus, m, nnb, box, left, right, count, clus2,
                         keep, ctr, dp, n, max_leaf);
      if ((err = hipcub::DeviceSelect::Flagged(stmp, stmp_bytes, clus2, keep, clus, nsel, m, s))) break;
      int mm = 0;
      if ((err = hipMemcpyAsync(&mm, nsel, 4, hipMemcpyDeviceToHost, s)) || (err = hipStreamSynchronize(s))) break;
      if (mm >= m) err = hipErrorInvalidValue;  // no merge: cannot happen (the best pair is always mutual)
      m = mm;
    }
    uint32_t c[4];
    if (!err && !(err = hipMemcpyAsync(c, ctr, 16, hipMemcpyDeviceToHost, s)) && !(err = hipStreamSynchronize(s)) &&
        (c[0] != 0u || (c[3] & 0x80000000u)))
      err = hipErrorInvalidValue;  // not exactly n - 1 internal nodes
    pfree();
    if (err) return fail(err);
    afree(first, s);
    first = nullptr;  // PLOC subtrees are not key ranges: the collapse walks them
  } else {
    if ((err = hipMemsetAsync(parent, 0xFF, 4 * nn, s))) return fail(err);
    if (n > 1)
      hipLaunchKernelGGL(k_radix_tree, dim3(grid_of(n - 1)), dim3(kB), 0, s, keys2, n, left, right, parent, first,
                         count);
    if ((err = hipMemsetAsync(flag, 0, 4 * nn, s))) return fail(err);
    hipLaunchKernelGGL(k_boxes, dim3(grid_of(n)), dim3(kB), 0, s, tri, keys2, n, left, right, parent, box, flag, first,
                       count, dp, max_leaf);
  }
  // treelet restructuring passes (PRT_TRBVH; default 2 on the LBVH tree, 0 on PLOC's), then the collapse table over
  // the new topology.  Measured (scripts/gpu_trbvh.sh; C4 / Spaceship rate on the tree, build time):
  //   LBVH  0 / 1 / 2 / 3 passes: 2,997 / 3,364 / 3,529 / 3,537 Mrays/s (60 / 77 / 106 / 131 ms); ship 4,071 -> 4,372
  //   PLOC  0 / 1 / 2 / 3 passes: 3,514 / 3,532 / 3,525 / 3,533 Mrays/s (55 / 78 / 112 / 128 ms); ship 4,172 -> 4,402
  const char* tre = std::getenv("PRT_TRBVH");
  const int tr_passes = trbvh >= 0 ? trbvh : (tre ? std::atoi(tre) : (ploc ? 0 : 2));
  if (tr_passes > 0 && n >= 3) {
    float* tcost = nullptr;
    uint32_t* terr = nullptr;
    if ((err = hipMallocAsync(reinterpret_cast<void**>(&tcost), 4 * nn, s)) || (err = hipMallocAsync(reinterpret_cast<void**>(&terr), 4, s))) {
      afree(tcost, s);
      return fail(err);
    }
    auto tfree = [&]() { afree(tcost, s); afree(terr, s); };
    if ((err = hipMemsetAsync(terr, 0, 4, s))) { tfree(); return fail(err); }
    if (ploc) hipLaunchKernelGGL(k_parents, dim3(grid_of(n)), dim3(kB), 0, s, left, right, n, parent);
    for (int pass = 0; pass < tr_passes && !err; pass++) {
      if ((err = hipMemsetAsync(flag, 0, 4 * nn, s))) break;
      hipLaunchKernelGGL(k_trbvh, dim3(grid_of(n)), dim3(kB), 0, s, n, left, right, parent, box, count, tcost, flag,
                         terr);
    }
    if (!err && dp.C && !(err = hipMemsetAsync(flag, 0, 4 * nn, s)))
      hipLaunchKernelGGL(k_dp_rebuild, dim3(grid_of(n)), dim3(kB), 0, s, n, left, right, parent, box, count, flag, dp,
                         max_leaf, terr);
    uint32_t te = 0;
    if (!err && !(err = hipMemcpyAsync(&te, terr, 4, hipMemcpyDeviceToHost, s)) && !(err = hipStreamSynchronize(s)) &&
        te != 0u)
      err = hipErrorInvalidValue;  // malformed tree
    tfree();
    if (err) return fail(err);
    afree(first, s);
    first = nullptr;  // subtrees are no longer key ranges: the collapse walks them
  }
  // collapse, level by level from the binary root (node 0; the single leaf when n == 1)
  const Task t0{0, 0u};  // binary root: internal node 0, or the single leaf (node n - 1 = 0) when n == 1
  const uint32_t c0[4] = {1u, 0u, 0u, 0u};  // wide nodes used (the root), triangles used, next tasks
  if ((err = hipMemcpyAsync(ta, &t0, sizeof(Task), hipMemcpyHostToDevice, s)) ||
      (err = hipMemcpyAsync(ctr, c0, 16, hipMemcpyHostToDevice, s)))
    return fail(err);
  uint32_t ntasks = 1, depth = 0;
  if (level_ends) level_ends->assign(1, 1u);  // level 0: the root (node 0)
  while (ntasks) {
    depth++;
    const uint32_t zero = 0;
    if ((err = hipMemcpyAsync(ctr + 2, &zero, 4, hipMemcpyHostToDevice, s))) return fail(err);
    hipLaunchKernelGGL(k_collapse, dim3(grid_of(ntasks)), dim3(kB), 0, s, tri, keys2, n, left, right, box, first,
                       count, max_leaf, ta, ntasks, tb, ctr, nodes_out, tris_out, dp);
    if ((err = hipGetLastError())) return fail(err);
    uint32_t c[4];
    if ((err = hipMemcpyAsync(c, ctr, 16, hipMemcpyDeviceToHost, s)) || (err = hipStreamSynchronize(s)))
      return fail(err);
    if (c[3] & 0x80000000u) return fail(hipErrorInvalidValue);  // malformed tree (bounds checks above)
    ntasks = c[2];
    if (level_ends && ntasks) level_ends->push_back(c[0]);  // the nodes this level allocated: the next level
    std::swap(ta, tb);
    info->nodes = c[0];
    info->tris = c[1];
    info->leaves = c[3];
  }
  info->depth = (int32_t)depth;
  if (info->tris != (uint32_t)n) return fail(hipErrorInvalidValue);
  float rb[6];
  if ((err = hipMemcpyAsync(rb, box, 24, hipMemcpyDeviceToHost, s)) || (err = hipStreamSynchronize(s))) return fail(err);
  for (int k = 0; k < 3; k++) { info->bmin[k] = rb[k]; info->bmax[k] = rb[3 + k]; }
  return fail(hipSuccess);
}

hipError_t gpu_blas_finish(hipStream_t s, Node8* nodes, uint32_t n_nodes, uint32_t node_base, const TriMT* tris,
                           uint32_t n_tris, uint32_t tri_base, ShadeTri* stri, uint32_t prim_base) {
  if (n_nodes) hipLaunchKernelGGL(k_rebase, dim3(grid_of(n_nodes)), dim3(kB), 0, s, nodes, n_nodes, node_base, tri_base);
  if (n_tris)
    hipLaunchKernelGGL(k_prim_records, dim3(grid_of(n_tris)), dim3(kB), 0, s, tris, n_tris, tri_base, stri, prim_base);
  return hipGetLastError();
}

}  // namespace prt
