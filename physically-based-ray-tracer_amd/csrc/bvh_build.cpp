// bvh_build.cpp -- binned-SAH BLAS builder + SAH-optimal 8-wide collapse into the device layout (bvh_build.h).
#include "bvh_build.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
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
  // in double: boxes of extent above ~1e19 overflow a float area (and every SAH cost built on it)
  double area() const {
    const double e0 = (double)hi[0] - lo[0], e1 = (double)hi[1] - lo[1], e2 = (double)hi[2] - lo[2];
    if (e0 < 0 || e1 < 0 || e2 < 0) return 0.0;
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
  int nbins = kBins;  // SAH bins per axis (the instance BVH: 8, tinybvh's BVHBINS for its per-frame TLAS build)
  bool median = false;  // median splits on the widest centroid axis: a balanced tree of height ceil(log2 n)

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
    if (median) {
      if (count <= max_leaf) return;
      int ax = 0;
      for (int k = 1; k < 3; k++)
        if (cb.hi[k] - cb.lo[k] > cb.hi[ax] - cb.lo[ax]) ax = k;
      const int32_t mid = first + count / 2;
      std::nth_element(idx.begin() + first, idx.begin() + mid, idx.begin() + first + count, [&](uint32_t a, uint32_t c) {
        const float ca = cen[3 * (size_t)a + ax], cc = cen[3 * (size_t)c + ax];
        return ca < cc || (ca == cc && a < c);
      });
      emit_children(ni, first, count, mid, work);
      return;
    }
    // binned SAH over centroid bins (C_trav = 1, C_int = 1 per triangle); a pair that must split (the instance BVH's
    // one-instance leaves) has only the one split
    double best = 1e300;
    if (count == 2 && count > max_leaf) {
      emit_children(ni, first, count, first + 1, work);
      return;
    }
    int bax = -1, bsplit = -1;
    // the three axes' bins filled in one pass over the primitives (each primitive's box and centroid read once)
    const int nb = nbins;
    Box bins[3][kBins];
    int cnt[3][kBins] = {};
    float blo[3], bsc[3];
    bool live[3];
    for (int ax = 0; ax < 3; ax++) {
      blo[ax] = cb.lo[ax];
      live[ax] = cb.hi[ax] > cb.lo[ax];
      bsc[ax] = live[ax] ? nb / (cb.hi[ax] - cb.lo[ax]) : 0.0f;
      for (int k = 0; k < nb; k++) bins[ax][k].reset();
    }
    for (int32_t i = first; i < first + count; i++) {
      const uint32_t p = idx[i];
      const Box& pb = tb[p];
      const float* pc = &cen[3 * (size_t)p];
      for (int ax = 0; ax < 3; ax++) {
        if (!live[ax]) continue;
        const int k = std::min(nb - 1, std::max(0, (int)((pc[ax] - blo[ax]) * bsc[ax])));
        cnt[ax][k]++;
        bins[ax][k].grow(pb);
      }
    }
    for (int ax = 0; ax < 3; ax++) {
      if (!live[ax]) continue;
      double la[kBins - 1], ra[kBins - 1];
      int lc[kBins - 1], rc[kBins - 1];
      Box acc; acc.reset();
      int c = 0;
      for (int k = 0; k < nb - 1; k++) {
        if (cnt[ax][k]) acc.grow(bins[ax][k]);
        c += cnt[ax][k];
        la[k] = acc.area(); lc[k] = c;
      }
      acc.reset(); c = 0;
      for (int k = nb - 1; k > 0; k--) {
        if (cnt[ax][k]) acc.grow(bins[ax][k]);
        c += cnt[ax][k];
        ra[k - 1] = acc.area(); rc[k - 1] = c;
      }
      for (int k = 0; k < nb - 1; k++) {
        if (!lc[k] || !rc[k]) continue;
        const double cost = la[k] * lc[k] + ra[k] * rc[k];
        if (cost < best) { best = cost; bax = ax; bsplit = k; }
      }
    }
    const double parea = b.area();
    const double leaf_cost = (double)count;                     // C_int * n
    const double split_cost = parea > 0 ? 1.0 + best / parea : 1e300;  // C_trav + SAH
    if (count <= max_leaf && (bax < 0 || leaf_cost <= split_cost)) return;
    int32_t mid;
    if (bax < 0) {
      mid = first + count / 2;  // coincident centroids: split the range
    } else {
      const float lo = cb.lo[bax], sc = nbins / (cb.hi[bax] - lo);
      auto it = std::partition(idx.begin() + first, idx.begin() + first + count, [&](uint32_t p) {
        int k = std::min(nbins - 1, std::max(0, (int)((cen[3 * (size_t)p + bax] - lo) * sc)));
        return k <= bsplit;
      });
      mid = (int32_t)(it - idx.begin());
      if (mid == first || mid == first + count) mid = first + count / 2;
    }
    emit_children(ni, first, count, mid, work);
  }
  void emit_children(int32_t ni, int32_t first, int32_t count, int32_t mid, std::vector<int32_t>& work) {
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

// ---- spatial-split binary builder (SBVH: Stich, Friedrich, Dietrich 2009, "Spatial Splits in Bounding Volume
// Hierarchies"; what the reference's BVH::BuildHQ does, Core/tiny_bvh.h:1968-2284).  A node may split its
// references at a plane, cutting the triangles that straddle it: each side keeps the bounds of its part of the
// triangle (clipped against the plane, inside the reference's box), so a triangle can sit in several leaves.
// Spatial splits are tried only where the best object split's children overlap by more than alpha of the root
// area, and duplication stops once the references reach kSbvhSlack x the triangle count.  The output is the
// same binary tree form as Builder (nodes with children after their parent, leaf ranges of idx).
constexpr double kSbvhAlpha = 1e-5;
constexpr double kSbvhSlack = 1.5;

struct SpatialBuilder {
  struct Ref {
    uint32_t prim;
    Box box;
  };
  const float* tri = nullptr;
  int max_leaf = 3;
  size_t refs_total = 0, refs_cap = 0;
  double root_area = 0;
  std::vector<Node2>* nodes = nullptr;
  std::vector<uint32_t>* idx = nullptr;

  // bounds of the part of triangle `p` with lo <= x[ax] <= hi, intersected with `clip` (double arithmetic)
  Box clip_part(uint32_t p, int ax, double lo, double hi, const Box& clip) const {
    const float* a = tri + 12 * (size_t)p;
    double v[3][3];
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 3; k++) v[j][k] = a[4 * j + k];
    double blo[3] = {1e300, 1e300, 1e300}, bhi[3] = {-1e300, -1e300, -1e300};
    auto grow = [&](const double* q) {
      for (int k = 0; k < 3; k++) { blo[k] = std::min(blo[k], q[k]); bhi[k] = std::max(bhi[k], q[k]); }
    };
    for (int j = 0; j < 3; j++) {
      const double* P = v[j];
      const double* Q = v[(j + 1) % 3];
      if (P[ax] >= lo && P[ax] <= hi) grow(P);
      for (const double c : {lo, hi}) {
        if ((P[ax] < c && Q[ax] > c) || (P[ax] > c && Q[ax] < c)) {
          const double t = (c - P[ax]) / (Q[ax] - P[ax]);
          double X[3];
          for (int k = 0; k < 3; k++) X[k] = P[k] + t * (Q[k] - P[k]);
          X[ax] = c;
          grow(X);
        }
      }
    }
    Box b;
    for (int k = 0; k < 3; k++) {
      // outward rounding to float, then the reference's own box
      b.lo[k] = std::max(clip.lo[k], std::nextafter((float)blo[k], -3e38f));
      b.hi[k] = std::min(clip.hi[k], std::nextafter((float)bhi[k], 3e38f));
    }
    return b;
  }

  void build(int32_t T, std::vector<Node2>& out_nodes, std::vector<uint32_t>& out_idx) {
    nodes = &out_nodes;
    idx = &out_idx;
    std::vector<Ref> refs(T);
    Box root;
    root.reset();
    for (int32_t i = 0; i < T; i++) {
      const float* a = tri + 12 * (size_t)i;
      refs[i].prim = (uint32_t)i;
      refs[i].box.reset();
      refs[i].box.grow(a); refs[i].box.grow(a + 4); refs[i].box.grow(a + 8);
      root.grow(refs[i].box);
    }
    root_area = std::max(root.area(), 1e-30);
    refs_total = (size_t)T;
    refs_cap = (size_t)((double)T * kSbvhSlack);
    nodes->clear();
    nodes->reserve(2 * (size_t)T);
    idx->clear();
    nodes->push_back(Node2());
    struct Work { int32_t ni; std::vector<Ref> refs; };
    std::vector<Work> work;
    work.push_back({0, std::move(refs)});
    while (!work.empty()) {
      Work w = std::move(work.back());
      work.pop_back();
      split(w.ni, w.refs, work);
    }
  }

  template <class W>
  void split(int32_t ni, std::vector<Ref>& refs, W& work) {
    const int32_t count = (int32_t)refs.size();
    Box b, cb;
    b.reset(); cb.reset();
    for (const Ref& r : refs) {
      b.grow(r.box);
      float c[3];
      for (int k = 0; k < 3; k++) c[k] = 0.5f * (r.box.lo[k] + r.box.hi[k]);
      cb.grow(c);
    }
    (*nodes)[ni].box = b;
    // subtrees are finished depth first, so this node's leaves are idx[first, first + count) whatever its form
    (*nodes)[ni].first = (int32_t)idx->size();
    (*nodes)[ni].count = count;
    auto make_leaf = [&]() {
      for (const Ref& r : refs) idx->push_back(r.prim);
    };
    if (count <= 1) { make_leaf(); return; }
    // object split: binned SAH over the reference centroids
    double best = 1e300;
    int bax = -1, bsplit = -1;
    Box bl_best, br_best;
    for (int ax = 0; ax < 3; ax++) {
      const float lo = cb.lo[ax], hi = cb.hi[ax];
      if (!(hi > lo)) continue;
      Box bins[kBins];
      int cnt[kBins] = {0};
      for (int k = 0; k < kBins; k++) bins[k].reset();
      const float sc = kBins / (hi - lo);
      for (const Ref& r : refs) {
        const float c = 0.5f * (r.box.lo[ax] + r.box.hi[ax]);
        const int k = std::min(kBins - 1, std::max(0, (int)((c - lo) * sc)));
        cnt[k]++;
        bins[k].grow(r.box);
      }
      Box lacc[kBins - 1];
      int lc[kBins - 1];
      Box acc; acc.reset();
      int c = 0;
      for (int k = 0; k < kBins - 1; k++) {
        if (cnt[k]) acc.grow(bins[k]);
        c += cnt[k];
        lacc[k] = acc; lc[k] = c;
      }
      acc.reset(); c = 0;
      for (int k = kBins - 1; k > 0; k--) {
        if (cnt[k]) acc.grow(bins[k]);
        c += cnt[k];
        if (!lc[k - 1] || !c) continue;
        const double cost = lacc[k - 1].area() * lc[k - 1] + acc.area() * c;
        if (cost < best) { best = cost; bax = ax; bsplit = k - 1; bl_best = lacc[k - 1]; br_best = acc; }
      }
    }
    // spatial split: only where the object split's children overlap noticeably, within the duplication budget
    double sbest = 1e300;
    int sax = -1;
    double splane = 0;
    if (bax >= 0 && count > 2 * max_leaf && refs_total < refs_cap) {
      Box ov;
      for (int k = 0; k < 3; k++) { ov.lo[k] = std::max(bl_best.lo[k], br_best.lo[k]); ov.hi[k] = std::min(bl_best.hi[k], br_best.hi[k]); }
      if (ov.area() / root_area > kSbvhAlpha) {
        for (int ax = 0; ax < 3; ax++) {
          const double lo = b.lo[ax], hi = b.hi[ax], w = (hi - lo) / kBins;
          if (!(w > 0)) continue;
          Box bins[kBins];
          int enter[kBins] = {0}, leave[kBins] = {0};
          for (int k = 0; k < kBins; k++) bins[k].reset();
          auto bin_of = [&](double x) { return std::min(kBins - 1, std::max(0, (int)((x - lo) / w))); };
          for (const Ref& r : refs) {
            const int b0 = bin_of(r.box.lo[ax]), b1 = bin_of(r.box.hi[ax]);
            if (b0 == b1) {
              bins[b0].grow(r.box);
            } else {
              // binning prices the reference's box cut at the bin planes (the exact triangle clip is done only for
              // the chosen plane, below): an upper bound of each part, at a fraction of the cost
              for (int k = b0; k <= b1; k++) {
                Box part = r.box;
                if (k > b0) part.lo[ax] = std::max(part.lo[ax], (float)(lo + k * w));
                if (k < b1) part.hi[ax] = std::min(part.hi[ax], (float)(lo + (k + 1) * w));
                bins[k].grow(part);
              }
            }
            enter[b0]++;
            leave[b1]++;
          }
          Box lacc[kBins - 1];
          int lcnt[kBins - 1];
          Box acc; acc.reset();
          int c = 0;
          for (int k = 0; k < kBins - 1; k++) {
            acc.grow(bins[k]);
            c += enter[k];
            lacc[k] = acc; lcnt[k] = c;
          }
          acc.reset(); c = 0;
          for (int k = kBins - 1; k > 0; k--) {
            acc.grow(bins[k]);
            c += leave[k];
            if (!lcnt[k - 1] || !c || (lcnt[k - 1] == count && c == count)) continue;
            // the references this plane cuts must fit the remaining duplication budget
            if (refs_total + (size_t)(lcnt[k - 1] + c - count) > refs_cap) continue;
            const double cost = lacc[k - 1].area() * lcnt[k - 1] + acc.area() * c;
            if (cost < sbest) { sbest = cost; sax = ax; splane = lo + k * w; }
          }
        }
      }
    }
    const double parea = b.area();
    const double leaf_cost = (double)count;
    const double obj_cost = parea > 0 && bax >= 0 ? 1.0 + best / parea : 1e300;
    const double sp_cost = parea > 0 && sax >= 0 ? 1.0 + sbest / parea : 1e300;
    if (count <= max_leaf && leaf_cost <= std::min(obj_cost, sp_cost)) { make_leaf(); return; }
    std::vector<Ref> L, R;
    if (sax >= 0 && sp_cost < obj_cost) {
      // cut at splane: references entirely on one side stay whole, straddling ones are clipped into both
      const float s = (float)splane;
      for (const Ref& r : refs) {
        if (r.box.hi[sax] <= s) {
          L.push_back(r);
        } else if (r.box.lo[sax] >= s) {
          R.push_back(r);
        } else {
          Ref a = r, c = r;
          a.box = clip_part(r.prim, sax, -1e300, splane, r.box);
          c.box = clip_part(r.prim, sax, splane, 1e300, r.box);
          const bool ea = a.box.lo[0] <= a.box.hi[0] && a.box.lo[1] <= a.box.hi[1] && a.box.lo[2] <= a.box.hi[2];
          const bool ec = c.box.lo[0] <= c.box.hi[0] && c.box.lo[1] <= c.box.hi[1] && c.box.lo[2] <= c.box.hi[2];
          if (ea) L.push_back(a);
          if (ec) R.push_back(c);
          if (!ea && !ec) L.push_back(r);  // degenerate clip: keep the whole reference
          if (ea && ec) refs_total++;
        }
      }
      if (L.empty() || R.empty() || ((int32_t)L.size() == count && (int32_t)R.size() == count)) {
        L.clear(); R.clear();
        sax = -1;  // no progress: object split instead
      }
    }
    if (L.empty() && R.empty()) {
      if (bax < 0) {  // coincident centroids: halve the list
        L.assign(refs.begin(), refs.begin() + count / 2);
        R.assign(refs.begin() + count / 2, refs.end());
      } else {
        const float lo = cb.lo[bax], sc = kBins / (cb.hi[bax] - lo);
        for (const Ref& r : refs) {
          const float c = 0.5f * (r.box.lo[bax] + r.box.hi[bax]);
          const int k = std::min(kBins - 1, std::max(0, (int)((c - lo) * sc)));
          (k <= bsplit ? L : R).push_back(r);
        }
        if (L.empty() || R.empty()) {
          std::vector<Ref> all = std::move(L.empty() ? R : L);
          L.assign(all.begin(), all.begin() + count / 2);
          R.assign(all.begin() + count / 2, all.end());
        }
      }
    }
    std::vector<Ref>().swap(refs);
    const int32_t l = (int32_t)nodes->size();
    nodes->push_back(Node2());
    nodes->push_back(Node2());
    (*nodes)[ni].left = l;
    (*nodes)[ni].right = l + 1;
    work.push_back({l + 1, std::move(R)});
    work.push_back({l, std::move(L)});
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

namespace {

// per-axis power-of-two scale so that ext / 2^e <= 255; returns the biased exponent (e + 127)
// smallest biased exponent e with qmax * 2^(e-127) >= ext (the node grid step is a power of two, so
// origin + q * step and (origin - O) * rD + q * (step * rD) lose no precision in the step factor)
uint8_t grid_exponent(double ext, double qmax) {
  if (!(ext > 0)) return 1;
  int e = (int)std::ceil(std::log2(ext / qmax));
  while (std::ldexp(qmax, e) < ext) e++;
  while (e > -126 && std::ldexp(qmax, e - 1) >= ext) e--;
  return (uint8_t)std::min(254, std::max(1, e + 127));
}

// child-bound storage: 8-bit grid coordinates
struct Fmt8 {
  static constexpr double kQMax = 255.0;
  static void set(Node8& n, int s, const double* lo, const double* hi) {
    uint8_t* ql[3] = {&n.qlox[s], &n.qloy[s], &n.qloz[s]};
    uint8_t* qh[3] = {&n.qhix[s], &n.qhiy[s], &n.qhiz[s]};
    for (int k = 0; k < 3; k++) { *ql[k] = (uint8_t)lo[k]; *qh[k] = (uint8_t)hi[k]; }
  }
  static void empty(Node8& n, int s) {
    n.qlox[s] = n.qloy[s] = n.qloz[s] = 255;
    n.qhix[s] = n.qhiy[s] = n.qhiz[s] = 0;
  }
};
// SAH-optimal collapse of the binary tree into 8-wide nodes (Ylitie, Karras, Laine 2017, sec. 3.1, restated):
// C(n, i) = cheapest cost of representing binary subtree n by at most i slots of its parent, where one slot
// is either a leaf (<= max_leaf triangles, cost A(n) * c_tri * count) or a wide node (A(n) * c_node + the
// best distribution of its 8 slots over the two binary children).  Costs are area-weighted (SAH).
struct WideDp {
  std::vector<std::array<double, 9>> C;    // C[n][i], i = 1..8
  std::vector<std::array<int8_t, 9>> Dk;   // best left share k of D(n, j) = C(l, k) + C(r, j - k), j = 2..8
  std::vector<std::array<uint8_t, 9>> prev;  // C(n, i) == C(n, i - 1) (use fewer slots)
  std::vector<uint8_t> leaf1;              // the single-slot form of n is a leaf

  void compute(const Builder& B, float c_node, float c_tri) {
    const size_t N = B.nodes.size();
    C.assign(N, {});
    Dk.assign(N, {});
    prev.assign(N, {});
    leaf1.assign(N, 0);
    for (size_t n = N; n-- > 0;) {  // children are stored after their parent
      const Node2& x = B.nodes[n];
      const double A = std::max(x.box.area(), 1e-30);
      const double leafc = x.count <= B.max_leaf ? A * c_tri * (double)x.count : 1e300;
      if (x.leaf()) {
        for (int i = 1; i <= 8; i++) { C[n][i] = leafc; prev[n][i] = i > 1; }
        leaf1[n] = 1;
        continue;
      }
      double D[9];
      for (int j = 2; j <= 8; j++) {
        D[j] = 1e300;
        Dk[n][j] = 1;
        for (int k = 1; k < j; k++) {
          const double c = C[x.left][k] + C[x.right][j - k];
          if (c < D[j]) { D[j] = c; Dk[n][j] = (int8_t)k; }
        }
      }
      const double intc = A * c_node + D[8];
      leaf1[n] = leafc <= intc;
      C[n][1] = std::min(leafc, intc);
      for (int i = 2; i <= 8; i++) {
        prev[n][i] = C[n][i - 1] <= D[i];
        C[n][i] = prev[n][i] ? C[n][i - 1] : D[i];
      }
    }
  }
  // the slots (binary node ids) that subtree n occupies when given at most i slots
  void collect(const Builder& B, int32_t n, int i, int32_t* out, int& nc) const {
    if (i == 1 || B.nodes[n].leaf()) { out[nc++] = n; return; }
    if (prev[n][i]) { collect(B, n, i - 1, out, nc); return; }
    const int k = Dk[n][i];
    collect(B, B.nodes[n].left, k, out, nc);
    collect(B, B.nodes[n].right, i - k, out, nc);
  }
  // the <= 8 children of the wide node made from binary node n
  int expand(const Builder& B, int32_t n, int32_t* out) const {
    int nc = 0;
    if (B.nodes[n].leaf()) { out[nc++] = n; return nc; }
    const int k = Dk[n][8];
    collect(B, B.nodes[n].left, k, out, nc);
    collect(B, B.nodes[n].right, 8 - k, out, nc);
    return nc;
  }
};

// the fixed collapse of a median-split tree: every wide node takes the binary nodes three levels below it (or the
// leaves above that), so the wide tree has ceil(height / 3) levels (tlas8_median_depth)
struct LevelCollapse {
  const Builder* B;
  void collect(int32_t n, int lvl, int32_t* out, int& nc) const {
    if (lvl == 0 || B->nodes[n].leaf()) { out[nc++] = n; return; }
    collect(B->nodes[n].left, lvl - 1, out, nc);
    collect(B->nodes[n].right, lvl - 1, out, nc);
  }
  int expand(int32_t n, int32_t* out) const {
    int nc = 0;
    if (B->nodes[n].leaf()) { out[nc++] = n; return nc; }
    collect(B->nodes[n].left, 2, out, nc);
    collect(B->nodes[n].right, 2, out, nc);
    return nc;
  }
};

// relative SAH costs of an 8-wide node visit and of one triangle test in the traversal kernels
// (measured optimum on C4 at 1 : 1 with the persistent kernels)
constexpr float kWideNodeCost = 1.0f, kWideTriCost = 1.0f;  // tri cost swept 0.15-5 on C4: flat above 1

template <class NodeT, class Fmt, class Out>
void build_wide8(const float* triangles, int32_t T, int max_leaf, Out& out, bool spatial = false, int bins = kBins,
                 bool median = false) {
  Builder B;
  B.tri = triangles;
  B.nbins = bins;
  B.median = median;
  B.max_leaf = std::max(1, std::min(4, max_leaf));
  if (spatial) {
    SpatialBuilder SB;
    SB.tri = triangles;
    SB.max_leaf = B.max_leaf;
    SB.build(T, B.nodes, B.idx);
  } else {
    B.build(T);
  }
  for (int k = 0; k < 3; k++) { out.bmin[k] = B.nodes[0].box.lo[k]; out.bmax[k] = B.nodes[0].box.hi[k]; }
  out.tris.reserve(T);
  WideDp dp;  // the SAH-optimal collapse (round 1's greedy collapse: 2,636 against 3,529+ Mrays/s on C4, removed)
  const LevelCollapse lv{&B};  // (median trees)
  if (!median) dp.compute(B, kWideNodeCost, kWideTriCost);
  auto is_leaf = [&](int32_t n) { return median ? B.nodes[n].leaf() : dp.leaf1[n] != 0; };
  struct Item { int32_t n2; uint32_t n8; int depth; };
  std::vector<Item> work;
  out.nodes.push_back(NodeT());
  work.push_back({0, 0, 1});
  while (!work.empty()) {
    const Item it = work.back();
    work.pop_back();
    out.depth = std::max(out.depth, it.depth);
    int32_t ch[8];
    int nc = 0;
    nc = median ? lv.expand(it.n2, ch) : dp.expand(B, it.n2, ch);
    // inflated child boxes and the node grid
    float clo[8][3], chi[8][3];
    double nlo[3] = {1e300, 1e300, 1e300}, nhi[3] = {-1e300, -1e300, -1e300};
    for (int i = 0; i < nc; i++) {
      const Node2& c = B.nodes[ch[i]];
      for (int k = 0; k < 3; k++) { clo[i][k] = c.box.lo[k]; chi[i][k] = c.box.hi[k]; }
      inflate_box(clo[i], chi[i]);
      for (int k = 0; k < 3; k++) { nlo[k] = std::min(nlo[k], (double)clo[i][k]); nhi[k] = std::max(nhi[k], (double)chi[i][k]); }
    }
    // octant slot assignment: slot s holds the child that comes first for rays of octant s
    int child_in[8];
    for (int s = 0; s < 8; s++) child_in[s] = -1;
    {
      double pc[3];
      for (int k = 0; k < 3; k++) pc[k] = 0.5 * (nlo[k] + nhi[k]);
      double cost[8][8];
      for (int i = 0; i < nc; i++)
        for (int s = 0; s < 8; s++) {
          double d = 0;
          for (int k = 0; k < 3; k++) {
            const double cc = 0.5 * ((double)clo[i][k] + (double)chi[i][k]) - pc[k];
            d += ((s >> k) & 1) ? -cc : cc;
          }
          cost[i][s] = d;
        }
      bool used_c[8] = {false}, used_s[8] = {false};
      for (int n = 0; n < nc; n++) {
        double best = 1e300;
        int bi = -1, bs = -1;
        for (int i = 0; i < nc; i++)
          if (!used_c[i])
            for (int s = 0; s < 8; s++)
              if (!used_s[s] && cost[i][s] < best) { best = cost[i][s]; bi = i; bs = s; }
        used_c[bi] = used_s[bs] = true;
        child_in[bs] = bi;
      }
    }
    NodeT nd;
    std::memset(&nd, 0, sizeof(nd));
    nd.px = (float)nlo[0]; nd.py = (float)nlo[1]; nd.pz = (float)nlo[2];
    const double p[3] = {(double)nd.px, (double)nd.py, (double)nd.pz};
    uint8_t e[3];
    for (int k = 0; k < 3; k++) e[k] = grid_exponent(nhi[k] - p[k], Fmt::kQMax);
    nd.ex = e[0]; nd.ey = e[1]; nd.ez = e[2];
    const double sc[3] = {std::ldexp(1.0, (int)e[0] - 127), std::ldexp(1.0, (int)e[1] - 127),
                          std::ldexp(1.0, (int)e[2] - 127)};
    // interior children are stored contiguously in slot order; leaf triangles likewise
    nd.child_base = (uint32_t)out.nodes.size();
    nd.tri_base = (uint32_t)out.tris.size();
    uint32_t ninterior = 0;
    for (int s = 0; s < 8; s++)
      if (child_in[s] >= 0 && !is_leaf(ch[child_in[s]])) ninterior++;
    out.nodes.resize(out.nodes.size() + ninterior);
    uint32_t nextchild = nd.child_base, tri_off = 0;
    for (int s = 0; s < 8; s++) {
      const int i = child_in[s];
      if (i < 0) {  // empty slot: inverted box never hits
        Fmt::empty(nd, s);
        continue;
      }
      double qlo[3], qhi[3];
      for (int k = 0; k < 3; k++) {
        qlo[k] = std::min(Fmt::kQMax, std::max(0.0, std::floor(((double)clo[i][k] - p[k]) / sc[k])));
        qhi[k] = std::min(Fmt::kQMax, std::max(0.0, std::ceil(((double)chi[i][k] - p[k]) / sc[k])));
      }
      Fmt::set(nd, s, qlo, qhi);
      const Node2& c = B.nodes[ch[i]];
      if (is_leaf(ch[i])) {
        for (int32_t j = c.first; j < c.first + c.count; j++) {
          const uint32_t pr = B.idx[j];
          const float* a = triangles + 12 * (size_t)pr;
          TriMT t;
          for (int k = 0; k < 3; k++) {
            t.v0[k] = a[k];
            t.e1[k] = a[4 + k] - a[k];   // e1 = v1 - v0, e2 = v2 - v0 (tiny_bvh.h:4614-4616)
            t.e2[k] = a[8 + k] - a[k];
          }
          t.prim = pr; t.pad1 = 0; t.pad2 = 0;
          out.tris.push_back(t);
        }
        nd.meta[s] = (uint8_t)((tri_off << 3) | (uint32_t)c.count);
        tri_off += (uint32_t)c.count;
        out.leaves++;
      } else {
        nd.imask |= (uint8_t)(1u << s);
        work.push_back({ch[i], nextchild++, it.depth + 1});
      }
    }
    out.nodes[it.n8] = nd;
  }
}

}  // namespace

BuiltBlas8 build_blas8(const float* triangles, int32_t T, int max_leaf, bool spatial) {
  BuiltBlas8 out;
  build_wide8<Node8, Fmt8>(triangles, T, max_leaf, out, spatial);
  return out;
}

int tlas8_median_depth(int32_t n) {
  int h = 0;  // height of the median-split binary tree: ceil(log2 n)
  while (h < 31 && (int64_t(1) << h) < n) h++;
  return std::max(1, (h + 2) / 3);
}

BuiltTlas8 build_tlas8(const float* boxes, int32_t n, int max_depth) {
  // each instance box as a degenerate "triangle" {lo, hi, lo}: its bounds are the box, its centroid the box centre
  std::vector<float> fat(12 * (size_t)n, 0.0f);
  for (int32_t i = 0; i < n; i++) {
    const float* b = boxes + 6 * (size_t)i;
    float* t = fat.data() + 12 * (size_t)i;
    for (int k = 0; k < 3; k++) { t[k] = b[k]; t[4 + k] = b[3 + k]; t[8 + k] = b[k]; }
  }
  BuiltBlas8 w;
  build_wide8<Node8, Fmt8>(fat.data(), n, 1, w, false, 8);  // 8 bins: tinybvh's BVHBINS (Core/tiny_bvh.h:92-131)
  BuiltTlas8 out;
  if (max_depth > 0 && w.depth > max_depth) {  // deeper than the caller's stacks: the balanced tree instead
    w = BuiltBlas8();
    build_wide8<Node8, Fmt8>(fat.data(), n, 1, w, false, 8, true);
    out.median = true;
  }
  out.depth = w.depth;
  out.nodes = std::move(w.nodes);
  out.slot.assign(8 * out.nodes.size(), 0xFFFFFFFFu);
  for (size_t j = 0; j < out.nodes.size(); j++) {
    Node8& nd = out.nodes[j];
    for (int s = 0; s < 8; s++)
      if (!((nd.imask >> s) & 1u) && nd.meta[s]) out.slot[8 * j + s] = w.tris[nd.tri_base + (nd.meta[s] >> 3)].prim;
    nd.tri_base = (uint32_t)(8 * j);
  }
  return out;
}

}  // namespace prt
