// bvh_build.cpp -- binned-SAH BLAS builder + 4-wide collapse into the device layout (see bvh_build.h).
#include "bvh_build.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace prt {

namespace {

struct Box {
  float lo[3], hi[3];
  void reset() {
    for (int k = 0; k < 3; k++) { lo[k] = 1e30f; hi[k] = -1e30f; }
  }
  void grow(const float* p) {
    for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; k++) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
  }
  float area() const {
    float e0 = hi[0] - lo[0], e1 = hi[1] - lo[1], e2 = hi[2] - lo[2];
    if (e0 < 0 || e1 < 0 || e2 < 0) return 0.0f;
    return e0 * e1 + e1 * e2 + e2 * e0;
  }
};

struct Node2 {
  Box box;
  int32_t left = -1, right = -1;  // children (interior)
  int32_t first = 0, count = 0;   // leaf range in the index array
  bool leaf() const { return left < 0; }
};

constexpr int kBins = 32;

struct Builder {
  const float* tri;
  std::vector<Box> tb;
  std::vector<float> cen;  // 3 per tri
  std::vector<uint32_t> idx;
  std::vector<Node2> nodes;
  int max_leaf;

  void build(int32_t T) {
    tb.resize(T);
    cen.resize(3 * (size_t)T);
    idx.resize(T);
    for (int32_t i = 0; i < T; i++) {
      const float* a = tri + 12 * (size_t)i;
      tb[i].reset();
      tb[i].grow(a); tb[i].grow(a + 4); tb[i].grow(a + 8);
      for (int k = 0; k < 3; k++) cen[3 * (size_t)i + k] = 0.5f * (tb[i].lo[k] + tb[i].hi[k]);
      idx[i] = (uint32_t)i;
    }
    nodes.reserve(2 * (size_t)T);
    nodes.push_back(Node2());
    nodes[0].first = 0; nodes[0].count = T;
    std::vector<int32_t> work{0};
    while (!work.empty()) {
      int32_t ni = work.back();
      work.pop_back();
      split(ni, work);
    }
  }

  void split(int32_t ni, std::vector<int32_t>& work) {
    const int32_t first = nodes[ni].first, count = nodes[ni].count;
    Box b, cb;
    b.reset(); cb.reset();
    for (int32_t i = first; i < first + count; i++) {
      b.grow(tb[idx[i]]);
      cb.grow(&cen[3 * (size_t)idx[i]]);
    }
    nodes[ni].box = b;
    if (count <= 1) return;
    // binned SAH over centroid bins (C_trav = 1, C_int = 1 per triangle)
    float best = 1e30f;
    int bax = -1, bsplit = -1;
    for (int ax = 0; ax < 3; ax++) {
      const float lo = cb.lo[ax], hi = cb.hi[ax];
      if (!(hi > lo)) continue;
      Box bins[kBins];
      int cnt[kBins] = {0};
      for (int k = 0; k < kBins; k++) bins[k].reset();
      const float sc = kBins / (hi - lo);
      for (int32_t i = first; i < first + count; i++) {
        uint32_t p = idx[i];
        int k = std::min(kBins - 1, std::max(0, (int)((cen[3 * (size_t)p + ax] - lo) * sc)));
        cnt[k]++;
        bins[k].grow(tb[p]);
      }
      float la[kBins - 1], ra[kBins - 1];
      int lc[kBins - 1], rc[kBins - 1];
      Box acc; acc.reset();
      int c = 0;
      for (int k = 0; k < kBins - 1; k++) {
        if (cnt[k]) acc.grow(bins[k]);
        c += cnt[k];
        la[k] = acc.area(); lc[k] = c;
      }
      acc.reset(); c = 0;
      for (int k = kBins - 1; k > 0; k--) {
        if (cnt[k]) acc.grow(bins[k]);
        c += cnt[k];
        ra[k - 1] = acc.area(); rc[k - 1] = c;
      }
      for (int k = 0; k < kBins - 1; k++) {
        if (!lc[k] || !rc[k]) continue;
        float cost = la[k] * lc[k] + ra[k] * rc[k];
        if (cost < best) { best = cost; bax = ax; bsplit = k; }
      }
    }
    const float parea = b.area();
    const float leaf_cost = (float)count;                      // C_int * n
    const float split_cost = parea > 0 ? 1.0f + best / parea : 1e30f;  // C_trav + SAH
    if (count <= max_leaf && (bax < 0 || leaf_cost <= split_cost)) return;
    int32_t mid;
    if (bax < 0) {
      mid = first + count / 2;  // coincident centroids: split the range
    } else {
      const float lo = cb.lo[bax], sc = kBins / (cb.hi[bax] - lo);
      auto it = std::partition(idx.begin() + first, idx.begin() + first + count, [&](uint32_t p) {
        int k = std::min(kBins - 1, std::max(0, (int)((cen[3 * (size_t)p + bax] - lo) * sc)));
        return k <= bsplit;
      });
      mid = (int32_t)(it - idx.begin());
      if (mid == first || mid == first + count) mid = first + count / 2;
    }
    int32_t l = (int32_t)nodes.size();
    nodes.push_back(Node2());
    nodes.push_back(Node2());
    nodes[l].first = first; nodes[l].count = mid - first;
    nodes[l + 1].first = mid; nodes[l + 1].count = first + count - mid;
    nodes[ni].left = l; nodes[ni].right = l + 1;
    work.push_back(l + 1);
    work.push_back(l);
  }
};

}  // namespace

// Conservative inflation: the traversal must never cull a box that holds a triangle the MT test
// accepts (Moeller-Trumbore can accept points ~1 ulp outside the exact triangle).
void inflate_box(float* lo, float* hi) {
  for (int k = 0; k < 3; k++) {
    float ext = std::max(std::fabs(lo[k]), std::fabs(hi[k]));
    float pad = ext * 1e-6f + 1e-7f;
    lo[k] -= pad;
    hi[k] += pad;
  }
}

BuiltBlas build_blas(const float* triangles, int32_t T, int max_leaf) {
  BuiltBlas out;
  Builder B;
  B.tri = triangles;
  B.max_leaf = std::max(1, std::min(4, max_leaf));
  B.build(T);
  for (int k = 0; k < 3; k++) { out.bmin[k] = B.nodes[0].box.lo[k]; out.bmax[k] = B.nodes[0].box.hi[k]; }
  out.tris.reserve(T);

  // 4-wide collapse, depth-first.  Each entry: (node2 index, Node4 slot to fill).
  struct Item { int32_t n2; int32_t n4; int depth; };
  std::vector<Item> stack;
  out.nodes.push_back(Node4());
  stack.push_back({0, 0, 1});
  auto emit_leaf = [&](const Node2& n) -> uint32_t {
    uint32_t first = (uint32_t)out.tris.size();
    for (int32_t i = n.first; i < n.first + n.count; i++) {
      uint32_t p = B.idx[i];
      const float* a = triangles + 12 * (size_t)p;
      TriMT t;
      for (int k = 0; k < 3; k++) {
        t.v0[k] = a[k];
        t.e1[k] = a[4 + k] - a[k];   // e1 = v1 - v0, e2 = v2 - v0 (tiny_bvh.h:4614-4616)
        t.e2[k] = a[8 + k] - a[k];
      }
      t.prim = p; t.pad1 = 0; t.pad2 = 0;
      out.tris.push_back(t);
    }
    out.leaves++;
    return make_leaf(first, (uint32_t)n.count);
  };
  while (!stack.empty()) {
    Item it = stack.back();
    stack.pop_back();
    out.depth = std::max(out.depth, it.depth);
    // gather up to 4 children by opening the largest interior child
    int32_t ch[4];
    int nc = 0;
    const Node2& root = B.nodes[it.n2];
    if (root.leaf()) {
      ch[nc++] = it.n2;  // tiny mesh: root itself is a leaf -> single-leaf Node4
    } else {
      ch[nc++] = root.left;
      ch[nc++] = root.right;
      while (nc < 4) {
        int bi = -1;
        float ba = -1.0f;
        for (int i = 0; i < nc; i++) {
          const Node2& c = B.nodes[ch[i]];
          if (!c.leaf() && c.box.area() > ba) { ba = c.box.area(); bi = i; }
        }
        if (bi < 0) break;
        const Node2& c = B.nodes[ch[bi]];
        ch[bi] = c.left;
        ch[nc++] = c.right;
      }
    }
    Node4 nd;
    std::memset(&nd, 0, sizeof(nd));
    for (int i = 0; i < 4; i++) {
      if (i >= nc) {
        nd.lox[i] = nd.loy[i] = nd.loz[i] = 1e30f;   // empty slot: inverted box never hits
        nd.hix[i] = nd.hiy[i] = nd.hiz[i] = -1e30f;
        nd.child[i] = kEmptyChild;
        continue;
      }
      const Node2& c = B.nodes[ch[i]];
      float lo[3] = {c.box.lo[0], c.box.lo[1], c.box.lo[2]}, hi[3] = {c.box.hi[0], c.box.hi[1], c.box.hi[2]};
      inflate_box(lo, hi);
      nd.lox[i] = lo[0]; nd.loy[i] = lo[1]; nd.loz[i] = lo[2];
      nd.hix[i] = hi[0]; nd.hiy[i] = hi[1]; nd.hiz[i] = hi[2];
      if (c.leaf()) {
        nd.child[i] = emit_leaf(c);
      } else {
        int32_t slot = (int32_t)out.nodes.size();
        out.nodes.push_back(Node4());
        nd.child[i] = (uint32_t)slot;
        stack.push_back({ch[i], slot, it.depth + 1});
      }
    }
    out.nodes[it.n4] = nd;
  }
  return out;
}

}  // namespace prt
