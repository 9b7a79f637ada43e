// prt_wave2.hip -- the merged-trace wavefront path tracer for gfx950.
//
// The reference's recursive per-pixel Renderer::Trace (Core/Renderer.cpp:150-406) is re-cut into stages over
// queues of live work items.  One item = one pixel x reference frame; it traces its AA path pair
// sequentially, so the canonical RNG stream of SURVEY Appendix B is preserved.  All per-item state is SoA in
// HBM.  Queues are split into kNSub sub-queues, each with its own counter on its own 128-B line; appends are
// block-aggregated (one atomic per block), consumers read the kNSub counts into an LDS prefix table.
//
// Every random number of a path is drawn in the shading stage, so the shading
// of iteration i already knows the ray of iteration i+1 (the sampled bounce, or the AA path-2 primary
// ray when path 1 ends) and queues it at once.  The closest-hit rays of iteration i+1 and the shadow
// rays of iteration i are then traced by ONE persistent launch, and the NEE resolve of iteration i
// (which needs those shadow results) runs after it:
//
//   k_wave_init                                   P(0) = primary rays r1
//   for i = 0 .. iters:
//     k_trace2(i)    closest hits of P(i)  +  any hits of S(i-1)         (one launch, mixed lanes)
//     k_res2d(i)     the items of P(i-1) (rinfo kRiFresh), walked in index order: NEE result of iteration i-1,
//                    (result, throughput) stack, path end, frame write.  With the extensions or a debug render mode
//                    k_resmiss2(i) walks the queue P(i-1) instead and also shades, for the items k_shade2(i-1)
//                    queued into P(i) (a subset of P(i-1)), this iteration's misses (i = 0: k_miss2 over P(0))
//     k_shade2(i)    the sky radiance of the misses (no extensions), hit attributes, NEE set-up -> S(i), BRDF
//                    sample or path-2 start -> P(i+1)
//
// Hazards (all kernels on one stream): P(i+1) reuses P(i-1)'s buffer after the resolve (i) read it;
// S(i) reuses S(i-1)'s buffer after k_trace2(i) read it; the resolve (i) reads ne/nb/nk/vis/R/T of an item for
// iteration i-1 before it (misses) or k_shade2(i) (hits) overwrites them; rinfo keeps iteration i-1's status
// (and whether the item was queued) while info already holds the state of the queued next ray.
#include <cstdio>

#include "prt_launch.h"
#include "prt_path.h"
#include "prt_persist.h"
#include "prt_queue.h"

namespace prt {

#ifdef PRT_LANE_STATS  // diagnostic build: prt_persist.h lane counters, one 32-counter row per traversal launch
__device__ unsigned long long g_lane_stats[(kMaxIters + 2) * 32];
void lane_stats_dump() {
  static unsigned long long h[(kMaxIters + 2) * 32];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_lane_stats), sizeof(h)) != hipSuccess) return;
  for (int i = 0; i < kMaxIters + 2; i++) {
    const unsigned long long* r = h + 32 * i;
    if (!r[31]) continue;
    std::fprintf(stderr, "prt: lanestats %d", i);
    for (int k = 0; k < 32; k++) std::fprintf(stderr, " %llu", r[k]);
    std::fprintf(stderr, "\n");
  }
  static const unsigned long long z[(kMaxIters + 2) * 32] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lane_stats), z, sizeof(z));
}
#endif

// The resolve of the plain pipeline (no extensions, render mode 0) and of the merged one walks all items in index
// order and takes those whose rinfo carries kRiFresh (set by the shading of the last iteration, cleared by the
// resolve), so its record loads coalesce; with extensions or a debug render mode it walks the last iteration's queue
// (k_resmiss2), which also shades that iteration's misses
constexpr uint32_t kResFresh = kRiFresh;

// the merged pipeline's queue of path-2 primaries: the counters of iteration iters + 1 (kind 0), never a path queue
__device__ __forceinline__ uint32_t q2_iter(const TraceArgs& A) { return 2u * (uint32_t)A.bounces; }

// ---- init: items -> primary rays, appended to queue 0 (sub-queue = block % kNSub).  Merged pipeline (B.merge):
// the AA path-2 primary ray too (its jitter is drawn here, :61), into ro2 / rd2 and the path-2 queue Q2 (shq)
__global__ void __launch_bounds__(kBlock) k_wave_init(SceneDev S, TraceArgs A, TileMap M, WaveBufs B,
                                                      float4* __restrict__ out) {
  __shared__ uint32_t sm[8];
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* cnt = qcounter(B.ctr, 0, 0, sub);
  uint32_t* cnt2 = qcounter(B.ctr, q2_iter(A), 0, sub);
  for (uint32_t c = blockIdx.x; c * kBlock < B.n; c += gridDim.x) {
    const uint32_t i = c * kBlock + threadIdx.x;
    bool enq = false;
    if (i < B.n) {
      const uint32_t gi = B.base + i;  // item index within the call (batches cover consecutive ranges)
      const uint32_t f = gi / M.items, r = gi % M.items;
      int32_t x, y;
      const bool valid = item_pixel(M, r, x, y);
      if (valid && A.bounces > 0) {
        const uint32_t p = (uint32_t)(y * A.W + x);
        uint32_t seed = init_seed(A.seed + p + (uint32_t)A.W * (uint32_t)A.H * (A.frame_index + f));
        float jx = 0.0f, jy = 0.0f;
        if (A.flags & kAA) { jx = random_float(seed); jy = random_float(seed); }         // :61
        const Ray r1 = primary_ray(S, (float)x, (float)y, A.W, A.H);
        B.seed[i] = seed;
        B.jit[i] = make_float2(jx, jy);
        B.ro[i] = make_float4(r1.O.x, r1.O.y, r1.O.z, 0.0f);
        B.rd[i] = make_float4(r1.D.x, r1.D.y, r1.D.z, 0.0f);
        B.info[i] = 0u;
        B.s1[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);
        if (B.merge) {
          const Ray r2 = primary_ray(S, (float)x + jx, (float)y + jy, A.W, A.H);
          B.ro2[i] = make_float4(r2.O.x, r2.O.y, r2.O.z, 0.0f);
          B.rd2[i] = make_float4(r2.D.x, r2.D.y, r2.D.z, 0.0f);
          B.rinfo[B.n + i] = 0u;
        }
        B.rinfo[i] = 0u;
        enq = true;
      } else {
        out[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);  // bounces == 0: Trace returns 0, t1 stays BVH_FAR
        if (B.merge) B.rinfo[B.n + i] = 0u;
        B.rinfo[i] = 0u;
      }
    }
    const uint32_t slot = block_append(cnt, enq ? 1u : 0u, sm);
    if (enq) B.q0[sub * B.qcap + slot] = i;
    if (B.merge) {
      const uint32_t s2 = block_append(cnt2, enq ? 1u : 0u, sm);
      if (enq) B.shq[sub * B.scap + s2] = i;
    }
  }
}

// ---- a shadow-queue entry (light << 29 | index) -> its world ray: rebuilt by light_ray from the item's hit point
// (hp, one per item for its up to four light-class rays) exactly as the shading kernel's NEE built it; the area
// light's rays (EXT, light kLightArea, index = item) are stored whole in ao / ad
constexpr uint32_t kShIndexMask = (1u << 29) - 1u;
__device__ __forceinline__ void shadow_of(const SceneDev& S, const WaveBufs& B, uint32_t code, V3& O, V3& D,
                                          float& tmax) {
  const uint32_t light = code >> 29;
  if (light == kLightArea) {
    const float4 o = B.ao[code & kShIndexMask], d = B.ad[code & kShIndexMask];
    O = v3(o.x, o.y, o.z);
    D = v3(d.x, d.y, d.z);
    tmax = o.w;
    return;
  }
  const float4 I = B.hp[(code & kShIndexMask) >> 2];
  Ray r;
  V3 L;
  float dl;
  light_ray(S, light, v3(I.x, I.y, I.z), r, tmax, L, dl);
  O = r.O;
  D = r.D;
}
// the visibility byte of a shadow-queue entry: 4 x item + k, or 4n + item for the area light's ray
__device__ __forceinline__ uint32_t shadow_vis(const WaveBufs& B, uint32_t code) {
  return (code >> 29) == kLightArea ? 4u * B.n + (code & kShIndexMask) : (code & kShIndexMask);
}

// ---- one traversal launch: closest hits of P(iter) (iter < iters) + any hits of S(iter - 1) (iter > 0)
template <int REFILL, int STACK, int WAVES, int TAILN, bool TLAS, bool SPILL = false>
__global__ void __launch_bounds__(64, WAVES) k_trace2(SceneDev S, WaveBufs B, uint32_t iter, uint32_t iters) {
  __shared__ uint32_t lds_stack[2 * STACK * 64];
  __shared__ uint32_t prefP[kNSub + 1], prefS[kNSub + 1];
  __shared__ uint32_t tail_lds[tail_lds_words(TAILN)];
  uint8_t* vis8 = reinterpret_cast<uint8_t*>(B.vis);
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t nP = iter < iters ? load_prefix(B.ctr, iter, 0, prefP) : 0u;
  // merged pipeline, iteration 0: the second segment is the path-2 primaries (Q2, in shq; closest hits -> hit2)
  const bool q2 = iter == 0 && B.merge;
  const uint32_t nS = iter > 0 ? load_prefix(B.ctr, iter - 1, 1, prefS)
                               : (q2 ? load_prefix(B.ctr, iters + 1, 0, prefS) : 0u);
  const uint32_t total = nP + nS;
  if (blockIdx.x * 64u >= total) return;
  uint32_t* fctr = fetch_counters(B.ctr, iter, 0);
  uint32_t* dflag = fetch_counters(B.ctr, iter, 1);  // set once some wave found the queue empty (cleared per call)
  uint32_t part = xcc_id();
  // timeline diagnostic (s_memrealtime, one record per wave: start, first empty fetch, exit)
  unsigned long long* tl = B.tl ? B.tl + ((size_t)iter * kTlWaves + blockIdx.x) * 4 : nullptr;
  bool seen_drain = false;
  if (tl && threadIdx.x == 0) tl[0] = __builtin_amdgcn_s_memrealtime();
  trav8_persistent<2, STACK, REFILL, TAILN, TLAS, SPILL>(
      S, lds_stack + threadIdx.x,
      [&](uint32_t* base, uint32_t want) {
        const uint32_t got = fetch_some(fctr, total, part, base, want);
#ifdef PRT_DRAIN_POLL  // A/B: the first empty fetch of a wave tells the other waves
        if (got == 0 && !seen_drain && threadIdx.x == 0)
          __hip_atomic_store(dflag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (tl && got == 0 && !seen_drain) {
          seen_drain = true;
          if (threadIdx.x == 0) tl[1] = __builtin_amdgcn_s_memrealtime();
        }
        return got;
      },
      [&](uint32_t g, V3& O, V3& D, float& tmax, bool& any) -> uint32_t {
        float4 o, d;
        uint32_t h;
        if (g < nP) {
          h = q[map_slot(prefP, g, B.qcap)];
          o = B.ro[h];
          d = B.rd[h];
          tmax = kFar;
          any = false;
        } else if (q2) {  // a path-2 primary ray: handle = item | 1 << 31
          h = B.shq[map_slot(prefS, g - nP, B.scap)];
          o = B.ro2[h];
          d = B.rd2[h];
          tmax = kFar;
          any = false;
          h |= 0x80000000u;
        } else {
          h = map_slot(prefS, g - nP, B.scap);
          any = true;
          shadow_of(S, B, B.shq[h], O, D, tmax);
          return h;
        }
        O = v3(o.x, o.y, o.z);
        D = v3(d.x, d.y, d.z);
        return h;
      },
      [&](uint32_t h, bool any, V3& O, V3& D) {
        if (any) {
          float tmax;
          shadow_of(S, B, B.shq[h], O, D, tmax);
          return;
        }
        const bool p2 = (h & 0x80000000u) != 0u;
        const float4 o = p2 ? B.ro2[h & 0x7FFFFFFFu] : B.ro[h], d = p2 ? B.rd2[h & 0x7FFFFFFFu] : B.rd[h];
        O = v3(o.x, o.y, o.z);
        D = v3(d.x, d.y, d.z);
      },
      [&](uint32_t h, const Hit& hit, bool any, bool occluded) {
        if (any) {
          if (!occluded) vis8[shadow_vis(B, B.shq[h])] = 1;
        } else {
          const float4 rec = make_float4(hit.t, hit.u, hit.v, __uint_as_float(pack_hit(S, hit.prim, hit.inst)));
          if (h & 0x80000000u) B.hit2[h & 0x7FFFFFFFu] = rec;
          else B.hit[h] = rec;
        }
      },
      [&]() -> bool { return __hip_atomic_load(dflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u; },
#ifdef PRT_LANE_STATS
      B.coop_tail ? tail_lds : nullptr, g_lane_stats + 32 * iter);
#else
      B.coop_tail ? tail_lds : nullptr, tl ? tl + 3 : nullptr);
#endif
  if (tl && threadIdx.x == 0) tl[2] = __builtin_amdgcn_s_memrealtime();
}

// the skybox lookup out of line: its correctly rounded double atan2 / acos would otherwise raise the register
// budget of the shading kernel, which looks up the sky for its misses itself
// (the three fields it reads passed by value: a SceneDev& of a kernel argument would copy the struct to scratch)
__device__ __noinline__ V3 sample_sky_call(const float* sky, int32_t w, int32_t h, V3 D) {
  SceneDev S{};
  S.sky = sky;
  S.skyw = w;
  S.skyh = h;
  return sample_sky(S, D);
}

// ---- misses of P(iter) (:159): sky radiance (or 0) into ne, before k_shade2 replaces the ray.  EXT: a ray
// that reaches the area light before any geometry ends there (ne = its MIS-weighted radiance, hit = miss).
template <bool EXT>
__device__ __forceinline__ void miss_item(const SceneDev& S, const TraceArgs& A, const WaveBufs& B, uint32_t item) {
  float4 hh = B.hit[item];
  if constexpr (EXT) {
    if (S.area) {
      const float4 o = B.ro[item], d = B.rd[item];
      const AreaLight AL = area_light(S);
      float tq, cl;
      if (area_hit(AL, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), hh.x, tq, cl)) {
        const uint32_t depth = B.info[item] & 0xFFu;
        const float pdf = depth == 0 ? kFar : B.T[(size_t)(depth - 1) * B.n + item].w;
        const V3 L = area_seen(AL, tq, cl, pdf);
        B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
        B.hit[item] = make_float4(kFar, 0.0f, 0.0f, 0.0f);
        return;
      }
    }
  }
  if (hh.x < kFar) return;
  V3 L = v3(0.0f, 0.0f, 0.0f);
  if (A.flags & kSkybox) {
    const float4 d = B.rd[item];
    L = sample_sky_call(S.sky, S.skyw, S.skyh, v3(d.x, d.y, d.z));
  }
  B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
}
template <bool EXT>
__global__ void __launch_bounds__(kBlock) k_miss2(SceneDev S, TraceArgs A, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t pref[kNSub + 1];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    if (g >= total) continue;
    miss_item<EXT>(S, A, B, q[map_slot(pref, g, B.qcap)]);
  }
}

// the path of `item` ends at this iteration: with AA and path 1, queue path 2's primary ray (its jitter was
// drawn at init, :61) -- returns true when a ray was set up for P(iter + 1)
__device__ __forceinline__ bool start_path2(const SceneDev& S, const TraceArgs& A, const TileMap& M,
                                            const WaveBufs& B, uint32_t item, uint32_t path) {
  if (path != 0 || !(A.flags & kAA)) return false;
  const uint32_t r = (B.base + item) % M.items;
  int32_t x, y;
  item_pixel(M, r, x, y);
  const float2 j = B.jit[item];
  const Ray r2 = primary_ray(S, (float)x + j.x, (float)y + j.y, A.W, A.H);
  B.ro[item] = make_float4(r2.O.x, r2.O.y, r2.O.z, 0.0f);
  B.rd[item] = make_float4(r2.D.x, r2.D.y, r2.D.z, 0.0f);
  B.info[item] = 1u << 8;
  return true;
}

// the sub-path of `item` ends at this iteration (EXT): continue with the refraction ray of the deepest
// dielectric node whose reflection subtree this was (the reference's depth-first recursion order,
// Core/Renderer.cpp:346 before :358) -- returns true when a ray was set up for P(iter + 1)
__device__ __forceinline__ bool diel_next(const WaveBufs& B, uint32_t item, uint32_t depth, uint32_t path) {
  uint32_t ds = B.dst[item];
  const uint32_t pend = ds & ~(ds >> 8) & ~(ds >> 24) & 0xFFu & ((1u << depth) - 1u);
  if (!pend) return false;
  const uint32_t k = 31u - (uint32_t)__builtin_clz(pend);
  const float4 o = B.dro[(size_t)k * B.n + item], d = B.drd[(size_t)k * B.n + item];
  B.ro[item] = make_float4(o.x, o.y, o.z, 0.0f);
  B.rd[item] = make_float4(d.x, d.y, d.z, 0.0f);
  B.info[item] = (k + 1u) | (path << 8);
  B.dst[item] = ds | (1u << (8 + k));
  return true;
}

// ---- shading of P(iter): NEE set-up -> S(iter), BRDF sample or path-2 start -> P(iter + 1)
// k_shade2's parameter list as the kernarg segment holds it (explicit arguments in order, each at its natural
// alignment, as C lays out these members)
struct Shade2Args {
  SceneDev S;
  TraceArgs A;
  TileMap M;
  WaveBufs B;
  uint32_t iter;
};
typedef const __attribute__((address_space(4))) Shade2Args* Shade2ArgsPtr;
// EXT (area light, dielectrics): held to 3 waves/SIMD (167 VGPRs, no spills; unbounded it takes 175 and runs 2
// waves: C5 frame 135.7 -> 132.4 ms).  The plain form runs 4 waves at its natural 119 VGPRs (forcing 5 spilled
// and was 2 % slower).
template <bool EXT>
__global__ void __launch_bounds__(kBlock, EXT ? 3 : 1) k_shade2(SceneDev S, TraceArgs A, TileMap M, WaveBufs B, uint32_t iter) {
  const Shade2ArgsPtr args = (Shade2ArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  if (args->iter != iter || args->B.n != B.n) {  // the layout above does not match this compiler's: fail the call
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(S.diag + 1, 1u);
    return;
  }
  __shared__ uint32_t pref[kNSub + 1];
  __shared__ uint32_t sm[8];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  uint32_t* qn = (iter & 1) ? B.q0 : B.q1;
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* shcnt = qcounter(B.ctr, iter, 1, sub);
  uint32_t* ncnt = qcounter(B.ctr, iter + 1, 0, sub);
  uint32_t* shq = B.shq + (size_t)sub * B.scap;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  const uint32_t fl = A.flags;
  // software pipeline over the grid-stride chunks: the next chunk's item, info, hit and seed are loaded while this
  // chunk's item is shaded
  uint32_t item_n = 0, info_n = 0, seed_n = 0;
  float4 hh_n = make_float4(kFar, 0.0f, 0.0f, 0.0f);
  float4 ro_n = make_float4(0.0f, 0.0f, 0.0f, 0.0f), rd_n = ro_n;  // (plain form: the ray too)
  auto prefetch = [&](uint32_t cc) {
    const uint32_t gg = cc * kBlock + threadIdx.x;
    if (gg < total) {
      item_n = q[map_slot(pref, gg, B.qcap)];
      info_n = B.info[item_n];
      hh_n = B.hit[item_n];
      seed_n = B.seed[item_n];
      if (!EXT) { ro_n = B.ro[item_n]; rd_n = B.rd[item_n]; }
    }
  };
  prefetch(blockIdx.x);
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const float4 ro_c = ro_n, rd_c = rd_n;
    // The scene and buffer descriptors are read from the kernarg segment inside each chunk (scalar loads, scalar
    // cache) instead of being held in SGPRs across the loop: their ~90 live words spilled to VGPR lanes (378
    // v_readlane in the loop) when hoisted.  The empty asm hides the pointer's loop invariance.
    Shade2ArgsPtr ka = args;
    asm volatile("" : "+s"(ka));
    const SceneDev& Sc = *(const SceneDev*)&ka->S;
    const WaveBufs& Bc = *(const WaveBufs*)&ka->B;
    const uint32_t g = c * kBlock + threadIdx.x;
    uint32_t item = 0, info = 0, seed = 0, nr = 0;
    int kind = 0;
    float4 hh = make_float4(kFar, 0.0f, 0.0f, 0.0f);
    const bool active = g < total;
    if (active) {
      item = item_n; info = info_n; hh = hh_n;
      const uint32_t sd = seed_n;
      if ((info & 0x1FFu) == 0) Bc.s1[item].w = hh.x;                                        // r1.hit.t
      if (!EXT && hh.x >= kFar) {  // a miss (:159): the sky radiance (or 0) ends the path (EXT: k_miss2 / k_resmiss2)
        V3 L = v3(0.0f, 0.0f, 0.0f);
        if (fl & kSkybox) {
          const float4 d = EXT ? Bc.rd[item] : rd_c;
          L = sample_sky_call(Sc.sky, Sc.skyw, Sc.skyh, v3(d.x, d.y, d.z));
        }
        Bc.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
      }
      if (hh.x < kFar) {
        seed = sd;
        kind = nee_kind(fl, seed);                                                           // :198-214
        nr = (uint32_t)nee_rays(kind);
      }
    }
    prefetch(c + gridDim.x);
    const uint32_t s0 = block_append(shcnt, nr, sm);  // the block's shadow-ray slots, one atomic
    const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u;
    uint32_t status = kStMiss, emissive = 0;
    bool next = false;
    bool area_ray = false;
    if (nr) {
      const float4 o = EXT ? Bc.ro[item] : ro_c, d = EXT ? Bc.rd[item] : rd_c;
      const V3 D = v3(d.x, d.y, d.z);
      const uint32_t pk = __float_as_uint(hh.w);
      const V3 I = v3(o.x, o.y, o.z) + hh.x * D;                                             // tiny_bvh.h:586
      const V3 V = -D;
      const HitAttr ha = hit_attributes(Sc, hit_inst(Sc, pk), hit_prim(Sc, pk), hh.y, hh.z, (fl & kNormalMap) != 0);
      // a shadow ray is queued as (light, visibility index) with the item's hit point I stored once: the traversal
      // kernel rebuilds it (shadow_of)
      Bc.hp[item] = make_float4(I.x, I.y, I.z, 0.0f);
      float4 nk;
      const V3 brdf = nee_lights(Sc, fl, kind, I, V, ha.N, ha.m, seed, nk, [&](int k, uint32_t light) {
        shq[s0 + k] = (light << 29) | (4u * item + (uint32_t)k);
      });
      const V3 e = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * ha.m.emis;                // :196
      if (e.x != 0.0f || e.y != 0.0f || e.z != 0.0f) {  // otherwise e is +0 and the resolve rebuilds it
        Bc.ne[item] = make_float4(e.x, e.y, e.z, 0.0f);
        emissive = kRiEmissive;
      }
      Bc.nb[item] = make_float4(brdf.x, brdf.y, brdf.z, 0.0f);
      Bc.nk[item] = nk;
      Bc.vis[item] = 0u;
      status = kStNeeEnd;
      if constexpr (EXT) {
        // area-light sample (2 draws after the light-class NEE draws) at lit, non-delta, non-dielectric hits
        reinterpret_cast<uint8_t*>(Bc.vis)[4 * (size_t)Bc.n + item] = 0;
        if (Sc.area && (fl & kLighted) && ha.kind != kMatDielectric && !delta_lobe(ha.m)) {
          const float xi1 = random_float(seed), xi2 = random_float(seed);
          Ray sr;
          float tmax;
          V3 fa;
          if (area_nee(area_light(Sc), I, ha.N, V, ha.m, xi1, xi2, sr, tmax, fa)) {
            area_ray = true;
            Bc.ao[item] = make_float4(sr.O.x, sr.O.y, sr.O.z, tmax);
            Bc.ad[item] = make_float4(sr.D.x, sr.D.y, sr.D.z, 0.0f);
            Bc.na[item] = make_float4(fa.x, fa.y, fa.z, 0.0f);
          }
        }
      }
      if ((int)depth != A.bounces - 1) {                                                     // :329
        if (EXT && ha.kind == kMatDielectric) {                                              // :331-372
          const Dielectric dl = dielectric_split(I, D, ha.N);
          const size_t e = (size_t)depth * Bc.n + item;
          Bc.dro[e] = make_float4(dl.refr.O.x, dl.refr.O.y, dl.refr.O.z, dl.fresnel);
          Bc.drd[e] = make_float4(dl.refr.D.x, dl.refr.D.y, dl.refr.D.z, 0.0f);
          Bc.T[e] = make_float4(0.0f, 0.0f, 0.0f, kFar);  // w: the continuation is not BRDF-sampled
          const uint32_t bit = 1u << depth, keep = ~(0x01010101u << depth);
          Bc.dst[item] = (Bc.dst[item] & keep) | bit | (dl.has_refr ? 0u : (bit << 24));
          status = kStNeeCont;
          Bc.ro[item] = make_float4(dl.refl.O.x, dl.refl.O.y, dl.refl.O.z, 0.0f);
          Bc.rd[item] = make_float4(dl.refl.D.x, dl.refl.D.y, dl.refl.D.z, 0.0f);
          Bc.info[item] = (depth + 1u) | (path << 8);
          next = true;
        } else {
          V3 dir, thr;
          float bp = 2.0f;
          if (sample_bounce(ha.m, V, ha.N, seed, dir, thr, EXT ? &bp : nullptr)) {           // :376-399
            status = kStNeeCont;
            float pdf = 0.0f;
            if constexpr (EXT)  // MIS density of the sampled direction (kFar: delta lobe or no light sampling)
              pdf = (bp > 1.0f || !Sc.area || !(fl & kLighted)) ? kFar : brdf_pdf(ha.m, ha.N, V, dir, bp);
            Bc.T[(size_t)depth * Bc.n + item] = make_float4(thr.x, thr.y, thr.z, pdf);
            const Ray nr2 = make_ray(I + dir * kEpsilon, dir);                               // :404
            Bc.ro[item] = make_float4(nr2.O.x, nr2.O.y, nr2.O.z, 0.0f);
            Bc.rd[item] = make_float4(nr2.D.x, nr2.D.y, nr2.D.z, 0.0f);
            Bc.info[item] = (depth + 1u) | (path << 8);
            next = true;
          }
        }
      }
      Bc.seed[item] = seed;
    }
    if constexpr (EXT) {  // the area-light shadow rays of the block, one more append
      const uint32_t a0 = block_append(shcnt, area_ray ? 1u : 0u, sm);
      if (area_ray) shq[a0] = (kLightArea << 29) | item;
    }
    if (active) {
      if (status != kStNeeCont) {
        if (EXT && Sc.has_diel) next = diel_next(Bc, item, depth, path);
        if (!next) next = start_path2(Sc, A, M, Bc, item, path);
      }
      Bc.rinfo[item] = depth | (path << 8) | (status << 16) | ((uint32_t)kind << 20) | (next ? kRiQueued : 0u) | emissive |
                       (EXT ? 0u : kResFresh);
    }
    const uint32_t slot = block_append(ncnt, next ? 1u : 0u, sm);
    if (next) qn[sub * Bc.qcap + slot] = item;
  }
}

// ---- merged pipeline (B.merge: AA, render mode 0, no extensions).  Shading of P(iter) as k_shade2<false>, each
// path's records (hit point, NEE record, status, (result, throughput) stack) in its own slot (slot = path, at
// slot * n + item), and where path 1 ends its item shades path 2's first segment at once, from the primary hit
// k_trace2(0) traced next to path 1's: the RNG stream continues from path 1's last draw exactly as if path 2's
// primary ray had been traced after path 1 ended, so the result is the same bit for bit and
// a frame needs one wavefront iteration (a traversal, a shading and a resolve launch) fewer.
__global__ void __launch_bounds__(kBlock, 1) k_shade2m(SceneDev S, TraceArgs A, TileMap M, WaveBufs B, uint32_t iter) {
  const Shade2ArgsPtr args = (Shade2ArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  if (args->iter != iter || args->B.n != B.n) {  // the Shade2Args layout does not match this compiler's: fail
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(S.diag + 1, 1u);
    return;
  }
  __shared__ uint32_t pref[kNSub + 1];
  __shared__ uint32_t sm[8];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  uint32_t* qn = (iter & 1) ? B.q0 : B.q1;
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* shcnt = qcounter(B.ctr, iter, 1, sub);
  uint32_t* ncnt = qcounter(B.ctr, iter + 1, 0, sub);
  uint32_t* shq = B.shq + (size_t)sub * B.scap;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  const uint32_t fl = A.flags;
  const uint32_t levels = (uint32_t)max(1, A.bounces - 1);
  uint32_t item_n = 0, info_n = 0, seed_n = 0;
  float4 hh_n = make_float4(kFar, 0.0f, 0.0f, 0.0f);
  auto prefetch = [&](uint32_t cc) {
    const uint32_t gg = cc * kBlock + threadIdx.x;
    if (gg < total) {
      item_n = q[map_slot(pref, gg, B.qcap)];
      info_n = B.info[item_n];
      hh_n = B.hit[item_n];
      seed_n = B.seed[item_n];
    }
  };
  prefetch(blockIdx.x);
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    Shade2ArgsPtr ka = args;  // descriptors from the kernarg segment per chunk (k_shade2)
    asm volatile("" : "+s"(ka));
    const SceneDev& Sc = *(const SceneDev*)&ka->S;
    const WaveBufs& Bc = *(const WaveBufs*)&ka->B;
    const uint32_t g = c * kBlock + threadIdx.x;
    const bool active = g < total;
    uint32_t item = 0, info = 0, seed = 0;
    float4 hh = make_float4(kFar, 0.0f, 0.0f, 0.0f);
    if (active) { item = item_n; info = info_n; hh = hh_n; seed = seed_n; }
    prefetch(c + gridDim.x);
    bool next = false, need2 = false;
#pragma unroll 1
    for (int pass = 0; pass < 2; pass++) {
      const bool act = pass == 0 ? active : need2;
      if (pass == 1 && act) { info = 1u << 8; hh = Bc.hit2[item]; }          // path 2, depth 0: its primary hit
      const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u;
      const size_t sn = (size_t)path * Bc.n + item;                         // this path's record slot
      const float4* rop = pass ? Bc.ro2 : Bc.ro;
      const float4* rdp = pass ? Bc.rd2 : Bc.rd;
      int kind = 0;
      uint32_t nr = 0;
      if (act) {
        if ((info & 0x1FFu) == 0) Bc.s1[item].w = hh.x;                                     // r1.hit.t
        if (hh.x >= kFar) {  // a miss (:159): the sky radiance (or 0) ends the path
          V3 L = v3(0.0f, 0.0f, 0.0f);
          if (fl & kSkybox) {
            const float4 d = rdp[item];
            L = sample_sky_call(Sc.sky, Sc.skyw, Sc.skyh, v3(d.x, d.y, d.z));
          }
          Bc.ne[sn] = make_float4(L.x, L.y, L.z, 0.0f);
        } else {
          kind = nee_kind(fl, seed);                                                        // :198-214
          nr = (uint32_t)nee_rays(kind);
        }
      }
      const uint32_t s0 = block_append(shcnt, nr, sm);  // the block's shadow-ray slots, one atomic per pass
      uint32_t status = kStMiss, emissive = 0;
      if (nr) {
        const float4 o = rop[item], d = rdp[item];
        const V3 D = v3(d.x, d.y, d.z);
        const uint32_t pk = __float_as_uint(hh.w);
        const V3 I = v3(o.x, o.y, o.z) + hh.x * D;                                           // tiny_bvh.h:586
        const V3 V = -D;
        const HitAttr ha = hit_attributes(Sc, hit_inst(Sc, pk), hit_prim(Sc, pk), hh.y, hh.z, (fl & kNormalMap) != 0);
        Bc.hp[sn] = make_float4(I.x, I.y, I.z, 0.0f);
        float4 nk;
        const V3 brdf = nee_lights(Sc, fl, kind, I, V, ha.N, ha.m, seed, nk, [&](int k, uint32_t light) {
          shq[s0 + k] = (light << 29) | (4u * (uint32_t)sn + (uint32_t)k);
        });
        const V3 e = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * ha.m.emis;                // :196
        if (e.x != 0.0f || e.y != 0.0f || e.z != 0.0f) {
          Bc.ne[sn] = make_float4(e.x, e.y, e.z, 0.0f);
          emissive = kRiEmissive;
        }
        Bc.nb[sn] = make_float4(brdf.x, brdf.y, brdf.z, 0.0f);
        Bc.nk[sn] = nk;
        Bc.vis[sn] = 0u;
        status = kStNeeEnd;
        if ((int)depth != A.bounces - 1) {                                                   // :329
          V3 dir, thr;
          if (sample_bounce(ha.m, V, ha.N, seed, dir, thr)) {                               // :376-399
            status = kStNeeCont;
            Bc.T[((size_t)path * levels + depth) * Bc.n + item] = make_float4(thr.x, thr.y, thr.z, 0.0f);
            const Ray nr2 = make_ray(I + dir * kEpsilon, dir);                               // :404
            Bc.ro[item] = make_float4(nr2.O.x, nr2.O.y, nr2.O.z, 0.0f);
            Bc.rd[item] = make_float4(nr2.D.x, nr2.D.y, nr2.D.z, 0.0f);
            Bc.info[item] = (depth + 1u) | (path << 8);
            next = true;
          }
        }
        Bc.seed[item] = seed;
      }
      if (act) {
        Bc.rinfo[sn] = depth | (path << 8) | (status << 16) | ((uint32_t)kind << 20) | emissive | kRiFresh;
        need2 = pass == 0 && path == 0 && status != kStNeeCont && (fl & kAA);
      }
    }
    const uint32_t slot = block_append(ncnt, next ? 1u : 0u, sm);
    if (next) qn[sub * Bc.qcap + slot] = item;
  }
}

// ---- debug render modes (:170-194): the hit's debug colour (or the sky) ends the path
__global__ void __launch_bounds__(kBlock) k_shade2_debug(SceneDev S, TraceArgs A, TileMap M, WaveBufs B,
                                                         uint32_t iter) {
  __shared__ uint32_t pref[kNSub + 1];
  __shared__ uint32_t sm[8];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  uint32_t* qn = (iter & 1) ? B.q0 : B.q1;
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* ncnt = qcounter(B.ctr, iter + 1, 0, sub);
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    bool next = false;
    uint32_t item = 0;
    if (g < total) {
      item = q[map_slot(pref, g, B.qcap)];
      const uint32_t info = B.info[item];
      const float4 hh = B.hit[item];
      if ((info & 0x1FFu) == 0) B.s1[item].w = hh.x;
      if (hh.x < kFar) {  // misses keep k_miss2's sky value
        const uint32_t pk = __float_as_uint(hh.w);
        const HitAttr ha = hit_attributes(S, hit_inst(S, pk), hit_prim(S, pk), hh.y, hh.z, (A.flags & kNormalMap) != 0);
        const V3 L = debug_view(S, A.mode, ha, hit_inst(S, pk), hit_prim(S, pk));
        B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
      }
      next = start_path2(S, A, M, B, item, (info >> 8) & 1u);
      B.rinfo[item] = (info & 0x1FFu) | (next ? kRiQueued : 0u);  // kStEndValue
    }
    const uint32_t slot = block_append(ncnt, next ? 1u : 0u, sm);
    if (next) qn[sub * B.qcap + slot] = item;
  }
}

// ---- NEE resolve of P(iter) (after k_trace2(iter + 1) traced S(iter)), stack, path end, frame write
template <bool EXT>
__device__ __forceinline__ void resolve_item(const SceneDev& S, const TraceArgs& A, const WaveBufs& B, uint32_t item,
                                             uint32_t ri, float4* __restrict__ out) {
  const uint32_t fl = A.flags;
  const uint32_t depth = ri & 0xFFu, path = (ri >> 8) & 1u, status = (ri >> 16) & 3u, kind = (ri >> 20) & 3u;
  // ne: the end value (miss, debug mode) or a hit's emissive term, stored only when nonzero (kRiEmissive)
  const bool nee = status == kStNeeEnd || status == kStNeeCont;
  const float4 ne = (!nee || (ri & kRiEmissive)) ? B.ne[item] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  V3 L = v3(ne.x, ne.y, ne.z);
  if (nee) {
    const float4 nb = B.nb[item], nk = B.nk[item];
    const uint32_t vw = B.vis[item];
    const uint32_t vis = ((vw & 0xFFu) ? 1u : 0u) | ((vw & 0xFF00u) ? 2u : 0u) | ((vw & 0xFF0000u) ? 4u : 0u) |
                         ((vw & 0xFF000000u) ? 8u : 0u);
    V3 result = nee_resolve(S, (int)kind, vis, L, v3(nb.x, nb.y, nb.z), nk, fl);
    if constexpr (EXT) {
      if (reinterpret_cast<const uint8_t*>(B.vis)[4 * (size_t)B.n + item]) {  // area light unoccluded
        const float4 a = B.na[item];
        result = result + v3(a.x, a.y, a.z);
      }
    }
    if (status == kStNeeCont) {  // the path goes on: result joins the stack
      B.R[(size_t)depth * B.n + item] = make_float4(result.x, result.y, result.z, 0.0f);
      return;
    }
    L = result;
  }
  if constexpr (EXT) {
    // unwind through dielectric nodes: the end of a reflection subtree parks its radiance in T[level] and
    // stops (the refraction subtree is already queued); the end of a refraction subtree combines (:369)
    uint32_t ds = S.has_diel ? B.dst[item] : 0u;
    bool parked = false;
    for (int k = (int)depth - 1; k >= 0; k--) {
      const size_t e = (size_t)k * B.n + item;
      const uint32_t bit = 1u << k;
      if (ds & bit) {
        const float F = B.dro[e].w;
        if (ds & (bit << 24)) {
          L = dielectric_combine(F, L, v3(0.0f, 0.0f, 0.0f));
        } else if (!(ds & (bit << 16))) {
          B.T[e] = make_float4(L.x, L.y, L.z, kFar);
          ds |= bit << 16;
          parked = true;
          break;
        } else {
          const float4 Lr = B.T[e];
          L = dielectric_combine(F, v3(Lr.x, Lr.y, Lr.z), L);
        }
        ds &= ~(0x01010101u << k);
        continue;
      }
      const float4 Rk = B.R[e], Tk = B.T[e];
      L = v3(Rk.x, Rk.y, Rk.z) + L * v3(Tk.x, Tk.y, Tk.z);
    }
    if (S.has_diel) B.dst[item] = ds;
    if (parked) return;
  } else {
    for (int k = (int)depth - 1; k >= 0; k--) {                                            // result + Trace(..) * throughput
      const float4 Rk = B.R[(size_t)k * B.n + item], Tk = B.T[(size_t)k * B.n + item];
      L = v3(Rk.x, Rk.y, Rk.z) + L * v3(Tk.x, Tk.y, Tk.z);
    }
  }
  const float4 s1 = B.s1[item];
  if (path == 0 && (fl & kAA)) {  // path 2 was queued by k_shade2; keep path 1's radiance
    B.s1[item] = make_float4(L.x, L.y, L.z, s1.w);
  } else {
    V3 res = (fl & kAA) ? 0.5f * (v3(s1.x, s1.y, s1.z) + L) : L;                           // :65
    if (fl & kGamma) res = v3(sqrtf(res.x), sqrtf(res.y), sqrtf(res.z));                  // :73-79
    out[item] = make_float4(res.x, res.y, res.z, s1.w);
  }
}
// ---- resolve of P(iter - 1) and the misses of P(iter) in one pass over P(iter - 1): P(iter) is the subset
// k_shade2(iter - 1) queued (rinfo bit kRiQueued), so each of its items is visited once, resolved first (it
// reads ne / T of iteration iter - 1) and then given its sky value (ne of iteration iter), the order of the
// separate kernels
template <bool EXT>
__global__ void __launch_bounds__(kBlock) k_resmiss2(SceneDev S, TraceArgs A, WaveBufs B, uint32_t iter,
                                                     uint32_t iters, uint32_t misses, float4* __restrict__ out) {
  __shared__ uint32_t pref[kNSub + 1];
  const uint32_t* q = ((iter - 1) & 1) ? B.q1 : B.q0;
  const uint32_t total = load_prefix(B.ctr, iter - 1, 0, pref);
  // software pipeline over the grid-stride chunks: the next chunk's item and rinfo are loaded while this
  // chunk's item is resolved
  uint32_t item_n = 0, ri_n = 0;
  auto prefetch = [&](uint32_t cc) {
    const uint32_t gg = cc * kBlock + threadIdx.x;
    if (gg < total) {
      item_n = q[map_slot(pref, gg, B.qcap)];
      ri_n = B.rinfo[item_n];
    }
  };
  prefetch(blockIdx.x);
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    const uint32_t item = item_n, ri = ri_n;
    prefetch(c + gridDim.x);
    if (g >= total) continue;
    resolve_item<EXT>(S, A, B, item, ri, out);
    if (misses && iter < iters && (ri & kRiQueued)) miss_item<EXT>(S, A, B, item);
  }
}

// dense resolve (plain pipeline, no extensions, render mode 0): every item in index order, the next item's rinfo
// loaded while this one is resolved
__global__ void __launch_bounds__(kBlock) k_res2d(SceneDev S, TraceArgs A, WaveBufs B, float4* __restrict__ out) {
  const uint32_t stride = gridDim.x * kBlock;
  uint32_t item = blockIdx.x * kBlock + threadIdx.x;
  uint32_t ri_n = item < B.n ? B.rinfo[item] : 0u;
  for (; item < B.n; item += stride) {
    const uint32_t ri = ri_n;
    if (item + stride < B.n) ri_n = B.rinfo[item + stride];
    if (!(ri & kRiFresh)) continue;
    resolve_item<false>(S, A, B, item, ri, out);
    B.rinfo[item] = ri & ~kRiFresh;
  }
}

// ---- merged pipeline: the resolve of P(iter - 1) per record slot (path 1's, then path 2's), as resolve_item<false>
__device__ __forceinline__ void resolve_slot(const SceneDev& S, const TraceArgs& A, const WaveBufs& B, uint32_t item,
                                             uint32_t path, uint32_t ri, float4* __restrict__ out) {
  const uint32_t fl = A.flags;
  const uint32_t levels = (uint32_t)max(1, A.bounces - 1);
  const size_t sn = (size_t)path * B.n + item;
  const uint32_t depth = ri & 0xFFu, status = (ri >> 16) & 3u, kind = (ri >> 20) & 3u;
  const bool nee = status == kStNeeEnd || status == kStNeeCont;
  const float4 ne = (!nee || (ri & kRiEmissive)) ? B.ne[sn] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  V3 L = v3(ne.x, ne.y, ne.z);
  if (nee) {
    const float4 nb = B.nb[sn], nk = B.nk[sn];
    const uint32_t vw = B.vis[sn];
    const uint32_t vis = ((vw & 0xFFu) ? 1u : 0u) | ((vw & 0xFF00u) ? 2u : 0u) | ((vw & 0xFF0000u) ? 4u : 0u) |
                         ((vw & 0xFF000000u) ? 8u : 0u);
    const V3 result = nee_resolve(S, (int)kind, vis, L, v3(nb.x, nb.y, nb.z), nk, fl);
    if (status == kStNeeCont) {  // the path goes on: result joins its stack
      B.R[((size_t)path * levels + depth) * B.n + item] = make_float4(result.x, result.y, result.z, 0.0f);
      return;
    }
    L = result;
  }
  for (int k = (int)depth - 1; k >= 0; k--) {                                              // result + Trace(..) * throughput
    const size_t e = ((size_t)path * levels + (uint32_t)k) * B.n + item;
    const float4 Rk = B.R[e], Tk = B.T[e];
    L = v3(Rk.x, Rk.y, Rk.z) + L * v3(Tk.x, Tk.y, Tk.z);
  }
  const float4 s1 = B.s1[item];
  if (path == 0 && (fl & kAA)) {  // path 2 follows (shaded in the same iteration); keep path 1's radiance
    B.s1[item] = make_float4(L.x, L.y, L.z, s1.w);
  } else {
    V3 res = (fl & kAA) ? 0.5f * (v3(s1.x, s1.y, s1.z) + L) : L;                           // :65
    if (fl & kGamma) res = v3(sqrtf(res.x), sqrtf(res.y), sqrtf(res.z));                  // :73-79
    out[item] = make_float4(res.x, res.y, res.z, s1.w);
  }
}
__global__ void __launch_bounds__(kBlock) k_res2md(SceneDev S, TraceArgs A, WaveBufs B, float4* __restrict__ out) {
  const uint32_t stride = gridDim.x * kBlock;
  uint32_t item = blockIdx.x * kBlock + threadIdx.x;
  uint32_t r0_n = 0, r1_n = 0;
  if (item < B.n) { r0_n = B.rinfo[item]; r1_n = B.rinfo[B.n + item]; }
  for (; item < B.n; item += stride) {
    const uint32_t r0 = r0_n, r1 = r1_n;
    if (item + stride < B.n) { r0_n = B.rinfo[item + stride]; r1_n = B.rinfo[B.n + item + stride]; }
    if (r0 & kRiFresh) {
      resolve_slot(S, A, B, item, 0u, r0, out);
      B.rinfo[item] = r0 & ~kRiFresh;
    }
    if (r1 & kRiFresh) {
      resolve_slot(S, A, B, item, 1u, r1, out);
      B.rinfo[B.n + item] = r1 & ~kRiFresh;
    }
  }
}

// LDS per wave (one block): 2 x STACK x 256 B of stack + 264 B of prefix tables + the tail slots, within
// 160 KB / (4 x WAVES) blocks per CU
#ifndef PRT_REFILL
#define PRT_REFILL 32  // idle lanes before a wave refills from the queue (A/B builds: -DPRT_REFILL=16 ...)
#endif
template <int STACK, int WAVES, int TAILN>
void launch_t2(const LaunchCfg& c, const SceneDev& S, const WaveBufs& B, uint32_t it, uint32_t iters) {
  static_assert(2 * STACK * 256 + 264 + 4 * 3 * TAILN <= 163840 / (4 * WAVES), "LDS over the occupancy budget");
  if (S.tlas)
    hipLaunchKernelGGL((k_trace2<PRT_REFILL, STACK, WAVES, TAILN, true>), dim3(256u * 4u * WAVES / c.groups), dim3(64), 0,
                       c.stream, S, B, it, iters);
  else
    hipLaunchKernelGGL((k_trace2<PRT_REFILL, STACK, WAVES, TAILN, false>), dim3(256u * 4u * WAVES / c.groups), dim3(64), 0,
                       c.stream, S, B, it, iters);
}
// persistent traversal occupancy (waves/SIMD) -> LDS stack groups per lane; a BVH deeper than the 18 LDS
// groups at 4 waves/SIMD hold runs the 4-wave form with the HBM spill columns (S.spill)
static void launch_trace2(const LaunchCfg& c, const SceneDev& S, const WaveBufs& B, uint32_t it, uint32_t iters) {
  if (S.spill) {
    if (S.tlas)
      hipLaunchKernelGGL((k_trace2<32, 18, 4, 32, true, true>), dim3(kSpillTraceBlocks / c.groups), dim3(64), 0,
                         c.stream, S, B, it, iters);
    else
      hipLaunchKernelGGL((k_trace2<32, 18, 4, 32, false, true>), dim3(kSpillTraceBlocks / c.groups), dim3(64), 0,
                         c.stream, S, B, it, iters);
  } else if (c.occ == 7) launch_t2<9, 7, 64>(c, S, B, it, iters);
  else if (c.occ == 6) launch_t2<11, 6, 64>(c, S, B, it, iters);
  else if (c.occ == 5) launch_t2<14, 5, 32>(c, S, B, it, iters);
  else launch_t2<18, 4, 32>(c, S, B, it, iters);
}

// producer grids (the kernels that append to the sub-queues: k_wave_init, the shading kernels): a multiple of kNSub,
// so that block b appends to sub-queue b % kNSub exactly the chunks c == b (mod kNSub) it consumes -- the bound
// ensure_wave sizes each sub-queue by (qcap).  1/groups of the resident blocks, rounded down to that multiple
__host__ inline unsigned producer_blocks(const LaunchCfg& c) {
  const unsigned g = 256u * 4u / c.groups;
  return g < kNSub ? kNSub : g - g % kNSub;
}

// one iteration of the merged pipeline: trace P(it) + S(it - 1), resolve P(it - 1), miss + shade P(it)
hipError_t launch_wave2_iter(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                             const WaveBufs& B, float4* out, WaveTimers* tm, uint32_t it) {
  if (B.n == 0) return hipSuccess;
  const unsigned gprod = producer_blocks(c);
  // k_shade2 over 4x the resident blocks when a call holds >= 2^21 items: the extra blocks queue behind the
  // resident ones and even out the kernel's end (C4 frame -1 to -2 %); below that the extra launch width costs
  // more than it evens out (world-8 shares). PRT_SHADE_GRID overrides (A/B runs).
#ifndef PRT_SHADE_GRID
  const unsigned gshade = B.n >= (1u << 21) ? 4u * gprod : gprod;
#else
  // the sub-queue bound of ensure_wave (qcap) holds only when block b appends to sub-queue b % kNSub for
  // chunks c == b (mod kNSub), i.e. for grids that are multiples of kNSub
  static_assert(PRT_SHADE_GRID % kNSub == 0, "PRT_SHADE_GRID must be a multiple of kNSub");
  const unsigned gshade = PRT_SHADE_GRID;
#endif
  const uint32_t iters = wave_iters(S.has_diel != 0, A.bounces, A.flags, B.merge != 0);
  if (tm) (void)hipEventRecord(tm->ev[4 * it + 0], c.stream);
  launch_trace2(c, S, B, it, iters);
  if (tm) (void)hipEventRecord(tm->ev[4 * it + 1], c.stream);
  const bool ext = (S.area || S.has_diel) && A.mode == 0;
  // the misses' sky radiance: by k_shade2<false> itself, or (extensions: the area light can turn a hit into a miss
  // first; debug render modes) by k_miss2 / k_resmiss2 before the shading
  const uint32_t sep_miss = (ext || A.mode != 0) ? 1u : 0u;
#ifndef PRT_RES_GRID
  const unsigned gres = gprod;
#else
  const unsigned gres = PRT_RES_GRID;  // A/B
#endif
  // the dense resolves over 2x the resident producer blocks (8 waves/SIMD), at most one chunk per block
  const unsigned gdense = std::min<unsigned>(2u * gprod, (B.n + kBlock - 1) / kBlock);
  if (it > 0 && B.merge) {
    hipLaunchKernelGGL(k_res2md, dim3(gdense), dim3(kBlock), 0, c.stream, S, A, B, out);
  } else if (it > 0 && !ext && !sep_miss) {
    hipLaunchKernelGGL(k_res2d, dim3(gdense), dim3(kBlock), 0, c.stream, S, A, B, out);
  } else if (it > 0) {  // resolve of P(it - 1) (+ misses of P(it)), one pass
    if (ext) hipLaunchKernelGGL(k_resmiss2<true>, dim3(gres), dim3(kBlock), 0, c.stream, S, A, B, it, iters, sep_miss,
                                out);
    else hipLaunchKernelGGL(k_resmiss2<false>, dim3(gres), dim3(kBlock), 0, c.stream, S, A, B, it, iters, sep_miss,
                            out);
  } else if (sep_miss) {
    if (ext) hipLaunchKernelGGL(k_miss2<true>, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, B, it);
    else hipLaunchKernelGGL(k_miss2<false>, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, B, it);
  }
  if (it < iters) {
    if (B.merge) hipLaunchKernelGGL(k_shade2m, dim3(gshade), dim3(kBlock), 0, c.stream, S, A, M, B, it);
    else if (A.mode != 0) hipLaunchKernelGGL(k_shade2_debug, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, M, B, it);
    else if (ext) hipLaunchKernelGGL(k_shade2<true>, dim3(gshade), dim3(kBlock), 0, c.stream, S, A, M, B, it);
    else hipLaunchKernelGGL(k_shade2<false>, dim3(gshade), dim3(kBlock), 0, c.stream, S, A, M, B, it);
  }
  if (tm) tm->iters = iters + 1;
  return hipGetLastError();
}

hipError_t launch_wave_init(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                            const WaveBufs& B, float4* out) {
  hipLaunchKernelGGL(k_wave_init, dim3(producer_blocks(c)), dim3(kBlock), 0, c.stream, S, A, M, B, out);
  return hipGetLastError();
}

}  // namespace prt
