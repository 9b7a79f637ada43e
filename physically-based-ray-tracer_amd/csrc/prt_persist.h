// prt_persist.h -- persistent-lane Node8 traversal for the wavefront queues (default traversal kernels).
//
// The lock-step loop of prt_traverse8.h runs a wave until its slowest of 64 rays is done, and every
// node visit waits for the lane with the most leaf triangles.  On the C4 secondary rays that leaves
// about a third of the lanes busy (scripts/trav_stats.cpp: lane efficiency 0.34 closest, 0.43 any-hit).
// Here every lane is a small state machine and one loop iteration does, per lane:
//   refill     lanes without a ray take the next queue entries (once >= kRefill lanes are idle; one
//              atomic per wave on an XCD-partitioned fetch counter, prt_queue.h)
//   instance   lanes done with a BLAS enter the next instance whose world box the ray hits (TLAS loop)
//   node       lanes with no pending triangles visit one Node8 node (8 quantised child slabs), keep its
//              hit leaf children as pending and step to the next interior child / pop the LDS stack
//   triangle   lanes with pending leaf triangles test one of them (Moeller-Trumbore, prt_traverse.h)
// so node visits and triangle tests of different lanes share iterations instead of serialising.
// Results are those of blas_traverse8: the hit rule is order-independent (closest t, then smaller
// instance, then larger prim) and the box tests are conservative, so visiting order cannot change a hit.
//
// Cooperative tail (tail != nullptr).  Once the queue is drained a launch lasts as long as its slowest
// rays: a lone wave still spends ~0.5-1 us per iteration (a wave64 node visit is ~220 VALU), and the
// slowest rays take 100-200 iterations (scripts/trav_stats.cpp --dist), so the last waves leave
// 100-270 us after the queue emptied (PRT_DEBUG_QUEUES timeline).  When a drained wave holds
// <= kTailRays rays, its idle lanes become helpers: each takes a pending node group (the top of a
// walking lane's stack, or its remaining sibling group) and walks that subtree with the ray copied from
// the donor.  A team (owner + helpers) shares one LDS slot: helper count, best (t, prim) key, any-hit
// flag.  When the owner's own walk and all its helpers are done it merges the team's best hit --
// re-testing the winning triangle (ShadeTri.pad[0]) for its (u, v) -- and continues with the next
// instance or finishes.  The hit rule makes the split exact: the result does not depend on which lane
// visits which subtree.
//
#pragma once
#include "prt_traverse8.h"

namespace prt {

constexpr uint32_t kNoNode = 0xFFFFFFFFu;
constexpr uint32_t kInstGroup = 0x100u;  // gimask flag: the group's children are instances (TLAS walk)
// a drained wave with at most TAILN rays turns cooperative; its LDS: TAILN x {count | found << 16, key lo, key hi}
constexpr uint32_t tail_lds_words(int tailn) { return 3u * (uint32_t)tailn; }

// index of the n-th (0-based) set bit of m; n < popcount(m)
__device__ __forceinline__ uint32_t nth_set(uint64_t m, uint32_t n) {
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
    if (n >= c) { n -= c; m >>= w; pos += (uint32_t)w; }
  }
  return pos;
}

// Persistent traversal of one wave (blockDim.x == 64).  MODE 0: closest hit, 1: any hit, 2: each ray says
// (mixed queues).  Ray source and sink are callbacks:
//   fetch(uint32_t* base, uint32_t want) -> uint32_t got   (wave-uniform; called by all lanes)
//   load(uint32_t g, V3& O, V3& D, float& tmax, bool& any) -> handle   queue entry g -> world ray, a handle
//                                                                       and (MODE 2) its query kind
//   reload(uint32_t handle, bool any, V3& O, V3& D)        world ray again (next instance of the TLAS loop)
//   finish(uint32_t handle, const Hit& h, bool any, bool hit)  closest: h; any-hit: hit = occluded
//   tick(idle, drained)                                     wave-uniform, once at the top of every iteration:
//                                                           idle lanes, no refill coming (a hook for
//                                                           per-iteration bookkeeping; k_trace2 passes none)
// tail: tail_lds_words(TAILN) words of LDS for the cooperative tail, or nullptr (no tail mode).
// The world ray is not kept in registers (reloaded per extra instance) so the loop state fits the
// register budget of 6-8 waves/SIMD.
template <int MODE, int STACK, int REFILL, int TAILN = 32, bool TLAS = false, bool SPILL = false, class Fetch,
          class Load, class Reload, class Finish, class Tick, class Drained>
__device__ __forceinline__ void trav8_persistent_t(const SceneDev& S, uint32_t* __restrict__ stk, Fetch fetch,
                                                   Load load, Reload reload, Finish finish, Tick tick,
                                                   Drained drained_elsewhere, uint32_t* __restrict__ tail = nullptr,
                                                   unsigned long long* __restrict__ dbg = nullptr) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t lanes_below = (1ull << lane) - 1ull;
  bool active = false, drained = false;
  bool any = MODE == 1;
  uint32_t handle = 0;
  V3 O = v3(0.0f, 0.0f, 0.0f), D = v3(0.0f, 0.0f, 1.0f), rD = D;  // instance-space ray
  uint32_t oct = 0;
  Hit h;
  h.t = kFar; h.u = 0.0f; h.v = 0.0f; h.prim = 0; h.inst = 0;
  int inst = -1;
  uint32_t node = kNoNode, gbase = 0, gmask = 0, gimask = 0;
  int sp = 0;
  uint32_t* st = stk;  // the LDS stack column this lane walks with
  // SPILL: levels past STACK go to the lane's HBM spill column (BVHs deeper than the LDS stack holds)
  const LaneStack ls = lane_stack<STACK, 64>(S, stk);
  const int cap = SPILL ? ls.cap : STACK;
  auto put = [&](int lvl, uint32_t a, uint32_t b) {
    if (SPILL) {
      stack_put<STACK, 64>(ls, lvl, a, b);
    } else {
      st[(2 * lvl) * 64] = a;
      st[(2 * lvl + 1) * 64] = b;
    }
  };
  auto get = [&](int lvl, uint32_t& a, uint32_t& b) {
    if (SPILL) {
      stack_get<STACK, 64>(ls, lvl, a, b);
    } else {
      a = st[(2 * lvl) * 64];
      b = st[(2 * lvl + 1) * 64];
    }
  };
  uint32_t lhit = 0, ltri = 0, lmeta0 = 0, lmeta1 = 0, tcur = 0, tcnt = 0;  // pending leaf triangles
  bool found = false;  // tail: this lane improved its closest hit
  // TLAS walk (TLAS = true): O / D / rD / oct hold the world ray while inst < 0 and the instance ray while
  // inst >= 0.  Groups of the instance BVH sit on the same LDS stack below those of the BLAS being walked (tsp:
  // the stack level where that BLAS began); an instance group (kInstGroup in gimask) names instances by slot.
  int tsp = 0;
  auto set_ray = [&](const V3& Oi, const V3& Di) {
    O = Oi;
    D = Di;
    rD = v3(safercp(D.x), safercp(D.y), safercp(D.z));
    oct = (rD.x < 0.0f ? 1u : 0u) | (rD.y < 0.0f ? 2u : 0u) | (rD.z < 0.0f ? 4u : 0u);
  };
  // enter the first instance >= i0 whose world box the ray hits before h.t (tiny_bvh.h:2500-2565 TLAS
  // walk as a linear loop over <= kLinearInstances instance boxes); false when there is none.  TLAS: start
  // the instance-BVH walk at its root.
  auto enter = [&](int i0, const V3& Ow, const V3& Dw) -> bool {
    if constexpr (TLAS) {
      set_ray(Ow, Dw);
      inst = -1;
      node = 0;
      gmask = 0;
      sp = 0;
      tsp = 0;
      return true;
    } else {
      const V3 rDw = v3(safercp(Dw.x), safercp(Dw.y), safercp(Dw.z));
      int i = i0;
      while (i < S.ninst && slab1(S.inst[i].bmin, S.inst[i].bmax, Ow, rDw, h.t) >= kFar) i++;
      if (i >= S.ninst) return false;
      const InstDev& I = S.inst[i];
      inst = i;
      set_ray(xform_point(Ow, I.inv), xform_vector(Dw, I.inv));
      node = S.mesh[I.mesh].root;
      gmask = 0;
      sp = 0;
      return true;
    }
  };
  auto push_cur = [&]() {
    if (gmask && sp < cap) {
      put(sp, gbase, gmask | (gimask << 8));
      sp++;
    } else if (gmask) {
      stack_overflow(ls.ovf);
    }
  };
  // next child of the current group, or the next stacked group, or done with this BLAS (TLAS: with this BLAS,
  // or with the instance BVH when inst < 0).  TLAS: an instance child is entered here (world -> instance ray).
  auto next_node = [&]() {
    const int base = TLAS && inst >= 0 ? tsp : 0;
    if (!gmask && sp > base) {
      sp--;
      uint32_t m;
      get(sp, gbase, m);
      gmask = m & 0xFFu;
      gimask = m >> 8;
    }
    if (gmask) {
      const uint32_t bit = __builtin_ctz(gmask);
      gmask &= gmask - 1u;
      const uint32_t k = bit ^ oct;
      node = gbase + __builtin_popcount(gimask & ((1u << k) - 1u) & 0xFFu);
      if constexpr (TLAS) {
        if (gimask & kInstGroup) {
          const int id = (int)S.tlas_slot[node];
          push_cur();  // the remaining instances of the group
          tsp = sp;
          inst = id;
          const InstDev& I = S.inst[id];
          set_ray(xform_point(O, I.inv), xform_vector(D, I.inv));
          node = S.mesh[I.mesh].root;
          gmask = 0;
        }
      }
    } else {
      node = kNoNode;
    }
  };
  // interior children hit at a visited node: stack the rest of the current group, descend into the new one
  auto push_group = [&](uint32_t ihit, uint32_t imask, uint32_t child_base) {
    if (ihit) {
      push_cur();
      gbase = child_base;
      gmask = order_mask(ihit, oct);
      gimask = imask;
    }
    next_node();
  };
  // leave the BLAS of instance `inst` (its walk and triangle tests done): the world ray again, then the next
  // instance-BVH child; false when the instance BVH is done too
  auto leave_blas = [&]() -> bool {
    V3 Ow, Dw;
    reload(handle, any, Ow, Dw);
    set_ray(Ow, Dw);
    inst = -1;
    next_node();
    return node != kNoNode;
  };
  // one node visit (lanes without pending triangles)
  auto node_step = [&](float tlimit) {
    const bool top = TLAS && inst < 0;  // a node of the instance BVH
    const uint4* np = top ? reinterpret_cast<const uint4*>(S.tlas8 + node) : blas_node(S.nodes8, node);
    const uint4 a = np[0], b = np[1];
    const uint4 c = np[2], d = np[3], e = np[4];
    const uint32_t hits = node8_hits(a, c, d, e, O, rD, tlimit);
    const uint32_t imask = a.w >> 24;
    if (TLAS && top) {  // instance children: one group addressed by slot (tlas_slot[b.y + slot])
      const uint32_t ih = hits & imask, lh = hits & ~imask;
      if (ih) {
        push_cur();
        gbase = b.x; gmask = order_mask(ih, oct); gimask = imask;
      }
      if (lh) {
        push_cur();
        gbase = b.y; gmask = order_mask(lh, oct); gimask = 0xFFu | kInstGroup;
      }
      next_node();
      return;
    }
    lhit = hits & ~imask;
    ltri = b.y; lmeta0 = b.z; lmeta1 = b.w;
    push_group(hits & imask, imask, b.x);
  };
  // one triangle test (lanes with pending leaf triangles); returns true when an any-hit query hit
  auto tri_step = [&]() -> bool {
    if (tcnt == 0) {
      const uint32_t k = __builtin_ctz(lhit);
      lhit &= lhit - 1u;
      const uint32_t meta = ((k < 4 ? lmeta0 : lmeta1) >> (8 * (k & 3))) & 0xFFu;
      tcur = ltri + (meta >> 3);
      tcnt = meta & 7u;
    }
    float t, u, v;
    uint32_t prim;
    const bool hit = mt_test(S.tris + tcur, O, D, t, u, v, prim);
    tcur++;
    tcnt--;
    if (MODE == 1 || (MODE == 2 && any)) {
      if (hit && t < h.t) {  // tiny_bvh.h:6594 (h.t holds tmax)
        node = kNoNode; lhit = 0; tcnt = 0;
        return true;
      }
    } else if (hit && (t < h.t || (t == h.t && ((uint32_t)inst < h.inst ||
                                                ((uint32_t)inst == h.inst && prim > h.prim))))) {
      h.t = t; h.u = u; h.v = v; h.prim = prim; h.inst = (uint32_t)inst;
      found = true;
    }
    return false;
  };
#ifdef PRT_DRAIN_POLL
  uint32_t iter_no = 0;
#endif
#ifdef PRT_LANE_STATS  // diagnostic build: per-wave counters of how the lanes of each loop iteration are used,
                       // added to dbg[0..31] when the wave leaves (k_trace2: one 32-counter row per launch)
  uint32_t lst[32] = {};
  lst[31] = 1;
#endif
  while (true) {
    // ---- refill idle lanes from the queue
    const uint64_t idle = __ballot(!active);
    tick((uint32_t)__popcll(idle), drained);
#ifdef PRT_DRAIN_POLL  // A/B: learn of the empty queue from other waves (measured slower: DESIGN.md 6)
    if (tail && !drained && idle != 0 && (++iter_no & 3u) == 0 && drained_elsewhere()) drained = true;
#endif
    if (!drained && __popcll(idle) >= (uint32_t)REFILL) {
      uint32_t base = 0;
      const uint32_t want = (uint32_t)__popcll(idle);
      const uint32_t got = fetch(&base, want);
      if (got == 0) drained = true;
      if (!active) {
        const uint32_t rank = (uint32_t)__popcll(idle & lanes_below);
        if (rank < got) {
          V3 Ow, Dw;
          float tmax;
          bool a = MODE == 1;
          handle = load(base + rank, Ow, Dw, tmax, a);
          if (MODE == 2) any = a;
          h.t = tmax; h.u = 0.0f; h.v = 0.0f; h.prim = 0; h.inst = 0;
          lhit = 0; tcnt = 0;
          if (enter(0, Ow, Dw)) active = true;
          else finish(handle, h, any, false);
        }
      }
    }
    const uint64_t act = __ballot(active);
    if (act == 0) {
      if (drained) break;
      continue;
    }
    if (tail && drained && __popcll(act) <= (uint32_t)TAILN) break;  // cooperative tail below
#ifdef PRT_LANE_STATS
    {
      const uint32_t nn = (uint32_t)__popcll(__ballot(active && node != kNoNode && lhit == 0));
      const uint32_t nt = (uint32_t)__popcll(__ballot(active && (lhit | tcnt)));
      const uint32_t nd = (uint32_t)__popcll(__ballot(active && node == kNoNode && lhit == 0 && tcnt == 0));
      lst[0]++; lst[1] += (uint32_t)__popcll(act); lst[2] += nn; lst[3] += nt;
      lst[4] += nn ? 1u : 0u; lst[5] += nt ? 1u : 0u; lst[6] += (nn && nt) ? 1u : 0u; lst[7] += nd ? 1u : 0u;
      lst[8 + (nn + 7) / 8]++;
      lst[17 + (nt + 7) / 8]++;
    }
#endif
    // ---- BLAS done: next instance, or the ray is finished
    if (active && node == kNoNode && lhit == 0 && tcnt == 0) {
      bool more = false;
      if constexpr (TLAS) {
        if (inst >= 0) more = leave_blas();
      } else if (inst + 1 < S.ninst) {
        V3 Ow, Dw;
        reload(handle, any, Ow, Dw);
        more = enter(inst + 1, Ow, Dw);
      }
      if (!more) {
        finish(handle, h, any, false);
        active = false;
      }
    }
    // ---- one node visit for lanes whose leaf children have all been started: the remaining triangles of
    // the current leaf (tcur, tcnt) are tested alongside the next node visits (order-independent hit rule;
    // measured 1.5-2.5 % faster per launch on C4 than waiting for the leaf to finish)
    if (active && node != kNoNode && lhit == 0) node_step(h.t);
    // ---- one triangle test for lanes with pending leaf triangles
    if (active && (lhit | tcnt)) {
      if (tri_step()) {
        finish(handle, h, true, true);
        active = false;
      }
    }
  }
#ifdef PRT_LANE_STATS
  auto flush_stats = [&]() {
    if (dbg && lane == 0)
      for (int k = 0; k < 32; k++)
        if (lst[k]) atomicAdd(dbg + k, (unsigned long long)lst[k]);
  };
  if (__ballot(active) == 0) { flush_stats(); return; }
#else
  if (__ballot(active) == 0) return;
#endif

  if (tail) {
    // ---------------------------------------------------------------- cooperative tail
    // role: owner (active: holds the ray's handle) / helper (walks one subtree of an owner's ray) / free;
    // team slot of an owner = its rank among the owners at tail entry (< TAILN)
    // tstate: helpers still walking (low 16 bits) | any-hit: some team lane hit (kFoundBit)
    constexpr uint32_t kFoundBit = 1u << 16;
    uint32_t* tstate = tail;
    unsigned long long* tkey = reinterpret_cast<unsigned long long*>(tail + TAILN);  // best (t, ~prim)
    bool helper = false;
    uint32_t slot = (uint32_t)__popcll(__ballot(active) & lanes_below);
    if (active) {
      tstate[slot] = 0u;
      tkey[slot] = ~0ull;
    }
    found = false;
#ifdef PRT_TAIL_STATS  // diagnostic build (PRT_DEBUG_QUEUES timeline, word 3): owners at tail entry, tail
                       // iterations, tail entry time (s_memrealtime, low 32 bits)
    uint32_t ts_it = 0, ts_starve = 0, ts_full = 0, ts_hand = 0;
    const uint32_t ts_a0 = (uint32_t)__popcll(__ballot(active));
    const unsigned long long ts_t0 = __builtin_amdgcn_s_memrealtime();
    (void)ts_starve; (void)ts_full; (void)ts_hand;
#endif
    // an owner takes its helpers' best hit: (u, v) from the same triangle test on the same instance-space ray
    auto merge_team = [&]() {
      const unsigned long long k = tkey[slot];
      tkey[slot] = ~0ull;
      const float kt = __uint_as_float((uint32_t)(k >> 32));
      const uint32_t kp = ~(uint32_t)k;  // the key holds ~prim: the larger prim wins an equal t
      if (k != ~0ull && (kt < h.t || (kt == h.t && ((uint32_t)inst < h.inst ||
                                                   ((uint32_t)inst == h.inst && kp > h.prim))))) {
        const uint32_t g = S.stri[S.mesh[S.inst[inst].mesh].prim_base + kp].pad[0];
        float t, u, v;
        uint32_t prim;
        (void)mt_test(S.tris + g, O, D, t, u, v, prim);
        h.t = t; h.u = u; h.v = v; h.prim = prim; h.inst = (uint32_t)inst;
      }
    };
    while (true) {
      const bool member = active || helper;
      // an any-hit team that hit stops walking
      if (member && any && (tstate[slot] & kFoundBit)) { node = kNoNode; lhit = 0; tcnt = 0; }
      bool busy = member && (node != kNoNode || lhit != 0 || tcnt != 0);
      // ---- helpers done with their subtree: publish, leave the team
      if (helper && !busy) {
        if (!any && found) atomicMin(&tkey[slot], ((unsigned long long)__float_as_uint(h.t) << 32) | (~h.prim & 0xFFFFFFFFull));
        atomicSub(&tstate[slot], 1u);
        helper = false;
      }
      // ---- owners whose walk and helpers are done: merge, next instance or finish
      if (active && !busy) {
        const uint32_t ts = tstate[slot];
        const bool occl = any && (ts & kFoundBit);
        if (occl || (ts & 0xFFFFu) == 0u) {
          if (!any) merge_team();
          bool more = false;
          if constexpr (TLAS) {
            if (!occl && inst >= 0) more = leave_blas();
          } else if (!occl && inst + 1 < S.ninst) {
            V3 Ow, Dw;
            reload(handle, any, Ow, Dw);
            more = enter(inst + 1, Ow, Dw);
          }
          if (more) {
            busy = true;  // a closest query; no helper of this team is left
          } else {
            finish(handle, h, any, occl);
            active = false;
          }
        }
      }
      if (__ballot(active) == 0) break;  // helpers always belong to a live owner
#ifdef PRT_TAIL_STATS
      ts_it++;
#endif
      // ---- free lanes take a pending group from a walking lane: its top stack entry or its sibling group
      const uint64_t freem = __ballot(!active && !helper);
      // (TLAS: only groups of the BLAS being walked are handed out: a helper walks instance-space subtrees)
      const uint64_t donm = __ballot((active || helper) && busy && (!TLAS || inst >= 0) &&
                                     (sp > (TLAS ? tsp : 0) || gmask != 0) && !(any && (tstate[slot] & kFoundBit)));
#ifdef PRT_TAIL_STATS
      if (freem && !donm) ts_starve++;
      if (!freem && donm) ts_full++;
      if (freem && donm) ts_hand += min((uint32_t)__popcll(freem), (uint32_t)__popcll(donm));
#endif
      if (freem && donm) {
        const uint32_t npair = min((uint32_t)__popcll(freem), (uint32_t)__popcll(donm));
        uint32_t ub = 0, um = 0, ui = 0;
        if (((donm >> lane) & 1ull) && (uint32_t)__popcll(donm & lanes_below) < npair) {
          if (sp > (TLAS ? tsp : 0)) {
            sp--;
            uint32_t m;
            get(sp, ub, m);
            um = m & 0xFFu;
            ui = m >> 8;
          } else {
            ub = gbase; um = gmask; ui = gimask;
            gmask = 0;
          }
        }
        const uint32_t frank = (uint32_t)__popcll(freem & lanes_below);
        const bool take = ((freem >> lane) & 1ull) && frank < npair;
        const int src = (int)nth_set(donm, take ? frank : 0u);
        // every lane joins the shuffles (ds_bpermute); only the takers keep the values
        const float ox = __shfl(O.x, src), oy = __shfl(O.y, src), oz = __shfl(O.z, src);
        const float dx = __shfl(D.x, src), dy = __shfl(D.y, src), dz = __shfl(D.z, src);
        const float tt = __shfl(h.t, src);
        const int sinst = __shfl(inst, src), sany = __shfl((int)any, src);
        const uint32_t sslot = (uint32_t)__shfl((int)slot, src), shp = (uint32_t)__shfl((int)h.prim, src);
        const uint32_t shi = (uint32_t)__shfl((int)h.inst, src);
        const uint32_t sb = (uint32_t)__shfl((int)ub, src), sm = (uint32_t)__shfl((int)um, src);
        const uint32_t si = (uint32_t)__shfl((int)ui, src);
        if (take) {
          helper = true;
          O = v3(ox, oy, oz);
          D = v3(dx, dy, dz);
          rD = v3(safercp(D.x), safercp(D.y), safercp(D.z));
          oct = (rD.x < 0.0f ? 1u : 0u) | (rD.y < 0.0f ? 2u : 0u) | (rD.z < 0.0f ? 4u : 0u);
          inst = sinst;
          any = MODE == 1 || (MODE == 2 && sany != 0);
          slot = sslot;
          h.t = tt; h.prim = shp; h.inst = shi;
          gbase = sb; gmask = sm; gimask = si;
          sp = 0; tsp = 0; lhit = 0; tcnt = 0;
          found = false;
          next_node();
          atomicAdd(&tstate[slot], 1u);
          busy = true;
        }
      }
      // ---- one node visit / one triangle test per walking lane, as in the main loop
      // closest hit: boxes are culled against the team's best t so far (the owner's and every helper's hits
      // are published as they are found), not only this lane's; a box entered at exactly that t is still
      // visited, so ties still reach the hit rule
      float tlim = h.t;
      if (busy && !any) {
        const unsigned long long k = tkey[slot];
        if (k != ~0ull) tlim = fminf(tlim, __uint_as_float((uint32_t)(k >> 32)));
      }
#ifdef PRT_LANE_STATS
      {
        const uint32_t nn = (uint32_t)__popcll(__ballot(busy && node != kNoNode && lhit == 0 && tcnt == 0));
        const uint32_t nt = (uint32_t)__popcll(__ballot(busy && (lhit | tcnt)));
        lst[26]++; lst[27] += nn; lst[28] += nt; lst[29] += nn ? 1u : 0u; lst[30] += nt ? 1u : 0u;
      }
#endif
      if (busy && node != kNoNode && lhit == 0 && tcnt == 0) node_step(tlim);
      if (busy && (lhit | tcnt)) {
        const float t0 = h.t;
        const uint32_t p0 = h.prim;
        if (tri_step()) atomicOr(&tstate[slot], kFoundBit);
        if (!any && (h.t != t0 || h.prim != p0))
          atomicMin(&tkey[slot], ((unsigned long long)__float_as_uint(h.t) << 32) | (~h.prim & 0xFFFFFFFFull));
      }
    }
#ifdef PRT_TAIL_STATS
    if (dbg && lane == 0)
      *dbg = (unsigned long long)ts_a0 | ((unsigned long long)min(ts_it, 0xFFFFFFu) << 8) |
             ((unsigned long long)(uint32_t)ts_t0 << 32);
#endif
  }
#ifdef PRT_LANE_STATS
  flush_stats();
#endif
}

template <int MODE, int STACK, int REFILL, int TAILN = 32, bool TLAS = false, bool SPILL = false, class Fetch,
          class Load, class Reload, class Finish, class Drained>
__device__ __forceinline__ void trav8_persistent(const SceneDev& S, uint32_t* __restrict__ stk, Fetch fetch,
                                                 Load load, Reload reload, Finish finish, Drained drained_elsewhere,
                                                 uint32_t* __restrict__ tail = nullptr,
                                                 unsigned long long* __restrict__ dbg = nullptr) {
  trav8_persistent_t<MODE, STACK, REFILL, TAILN, TLAS, SPILL>(S, stk, fetch, load, reload, finish, [](uint32_t, bool) {},
                                                        drained_elsewhere, tail, dbg);
}

}  // namespace prt
