// prt_stream.hip -- the streaming path tracer: ONE persistent launch per call.
//
// The merged wavefront (prt_wave2.hip) runs a frame as 2 x bounces + 1 dependent traversal launches, each as long
// as its slowest ray: on a small share of a frame (one GPU's tiles of an 8-GPU node) those launch tails are most of
// the time.  Here nothing waits for a launch boundary.  An item (pixel x reference frame, the same
// items, RNG streams and arithmetic as prt_wave2.hip) moves between two queues:
//
//   ray queue    one entry per ray in flight: item << 3 | k (k < 4: shadow ray k of the item's last shading,
//                k = 4: its next closest-hit ray)
//   shade queue  items whose rays have all finished: the item's next visit resolves the NEE of its last shading
//                (Core/Renderer.cpp:216-310 with the shadow results), unwinds the (result, throughput) stack at a
//                path end (:376-405), then misses / shades the closest hit it just got (:159-399) and emits that
//                shading's rays -- or, with nothing left to trace, finishes the item
//
// Every wave of the persistent grid alternates a traversal phase (the persistent-lane loop of prt_persist.h:
// lanes refill from the ray queue and walk one node or test one triangle per iteration, until none of its lanes
// has a ray) and a shading phase (one item per lane), so the straggling rays of one bounce overlap the other
// items' shading and next bounces instead of idling the GPU.  The last finisher of an item's rays (an atomic on
// the item's pending word, which also collects the shadow rays' visibility bits) queues the item for shading.
//
// Queues: kParts partitions, one per XCD, each with a reservation counter (tail) and a claim counter (head).  Item
// i belongs to partition i % kParts for its whole life: its rays and its visits are queued there and only waves
// of that XCD (HW_REG_XCC_ID) claim from it.  Producers append with one atomic per wave and write entries;
// consumers claim tickets with one atomic per wave and poll their entries, resetting each after use.  A claim can
// run past the tail when waves race; that ticket's entry is written by a later append and its holder keeps
// polling it across phases, so no wave ever blocks on one.  A partition's waves leave when its live count is 0
// (every item finished), or at a time limit (error word set: the call fails).
//
// Coherence: the per-XCD L2 is coherent for every CU of its XCD, and an item never leaves its XCD inside the
// launch; a CU's L1 is not refreshed by other CUs' stores, so every load of mutable item state or of a queue word
// bypasses L1 (non-temporal / sc1 loads), and a writer drains its stores (s_waitcnt vmcnt(0)) before the atomic or
// queue entry that publishes them (MI355X_MICROARCH.md, inter-workgroup visibility).  Kernel boundaries hand the
// state over between calls.  Scene data (BVH, triangles, textures) is read-only and loaded plainly.
#include "prt_launch.h"
#include "prt_path.h"
#include "prt_persist.h"
#include "prt_queue.h"

namespace prt {

constexpr uint32_t kNoTk = 0xFFFFFFFFu;
constexpr uint32_t kRiFresh = 1u << 25;  // rinfo: the item's first visit (nothing to resolve yet)
constexpr int kStreamWaves = 4;          // waves / SIMD: the shading code needs 128 VGPRs
constexpr int kStreamStack = 18;         // LDS stack groups per lane at 4 waves (prt_wave2.hip launch_trace2)
constexpr uint32_t kStreamBlocks = 256u * 4u * kStreamWaves;
constexpr uint32_t kTkShift = 29;        // ticket = partition << 29 | index
constexpr unsigned long long kStreamLimit = 400000000ull;  // s_memrealtime ticks (100 MHz): 4 s

__device__ __forceinline__ uint32_t* ctl_at(uint32_t* ctl, uint32_t w) { return ctl + (size_t)w * kCtrStride; }
__device__ __forceinline__ uint32_t ld_rlx(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// control words are only ever changed by atomics: read them with one too (the value at the atomics' point of
// coherence, whatever copy a cache holds)
__device__ __forceinline__ uint32_t ld_ctl(uint32_t* p) { return atomicAdd(p, 0u); }
__device__ __forceinline__ void st_rlx(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// this wave's stores have completed (in uncached memory: visible to every reader) before what follows
#ifdef PRT_STREAM_FENCES  // diagnostic build: full agent-scope fences around every hand-off
__device__ __forceinline__ void drain_stores() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); }
#else
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void acquire() {}
#endif

// Loads of mutable item state: non-temporal loads, which bypass the CU's vector L1 (another CU's stores never
// refresh it) and are served by the XCD's L2 (MI355X_MICROARCH.md, inter-workgroup visibility).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 ld4(const float4* p) {
  const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 ld2(const float2* p) {
  const f2v v = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p));
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ uint32_t ld1(const uint32_t* p) { return __builtin_nontemporal_load(p); }

// shadow rays (bits 0-3 of the lanes' ray masks) of the wave, wave-uniform
__device__ __forceinline__ uint32_t nrays_w(uint32_t rays) {
  return (uint32_t)__popcll(__ballot(rays & 1u)) + (uint32_t)__popcll(__ballot(rays & 2u)) +
         (uint32_t)__popcll(__ballot(rays & 4u)) + (uint32_t)__popcll(__ballot(rays & 8u));
}

// wave-aggregated append of n (0..7) entries per lane to a queue partition: one atomic per wave; returns the lane's
// first index in the partition
__device__ __forceinline__ uint32_t wave_append(uint32_t* tail, uint32_t n) {
  const uint64_t b1 = __ballot(n & 1u), b2 = __ballot(n & 2u), b4 = __ballot(n & 4u);
  const uint64_t lt = (1ull << lane_id()) - 1ull;
  const uint32_t before = (uint32_t)__popcll(b1 & lt) + 2u * (uint32_t)__popcll(b2 & lt) + 4u * (uint32_t)__popcll(b4 & lt);
  const uint32_t tot = (uint32_t)__popcll(b1) + 2u * (uint32_t)__popcll(b2) + 4u * (uint32_t)__popcll(b4);
  uint32_t base = 0;
  if (lane_id() == 0 && tot) base = atomicAdd(tail, tot);
  return (uint32_t)__shfl((int)base, 0, 64) + before;
}

// wave-uniform claim of up to `want` tickets from partition p; returns the count, `first` the first ticket
__device__ __forceinline__ uint32_t claim(uint32_t* ctl, uint32_t tail_w, uint32_t head_w, uint32_t p, uint32_t want,
                                          uint32_t& first) {
  uint32_t got = 0, b = 0;
  if (lane_id() == 0) {
    const uint32_t t = ld_ctl(ctl_at(ctl, tail_w + p)), h = ld_ctl(ctl_at(ctl, head_w + p));
    if (t > h) {
      got = min(want, t - h);
      b = atomicAdd(ctl_at(ctl, head_w + p), got);
    }
  }
  got = (uint32_t)__shfl((int)got, 0, 64);
  first = (p << kTkShift) | (uint32_t)__shfl((int)b, 0, 64);
  return got;
}
// the entry of ticket tk, or kStreamEmpty while it is unwritten (consumed entries are reset for the next call)
__device__ __forceinline__ uint32_t take(uint32_t* q, uint32_t cap, uint32_t tk) {
  const uint32_t idx = tk & ((1u << kTkShift) - 1u);
  if (idx >= cap) return kStreamEmpty;  // past the capacity: never written (the producer raised the error word)
  uint32_t* e = q + (size_t)(tk >> kTkShift) * cap + idx;
  const uint32_t v = ld_rlx(e);
  if (v != kStreamEmpty) st_rlx(e, kStreamEmpty);
  return v;
}

// ---- items -> primary rays (k_wave_init's arithmetic, Core/Renderer.cpp:55-63)
__global__ void __launch_bounds__(kBlock) k_stream_init(SceneDev S, TraceArgs A, TileMap M, StreamBufs B,
                                                        float4* __restrict__ out) {
  for (uint32_t c = blockIdx.x; c * kBlock < B.n; c += gridDim.x) {
    const uint32_t i = c * kBlock + threadIdx.x;
    bool enq = false;
    if (i < B.n) {
      const uint32_t gi = B.base + i;
      const uint32_t f = gi / M.items, r = gi % M.items;
      int32_t x, y;
      const bool valid = item_pixel(M, r, x, y);
      if (valid && A.bounces > 0) {
        const uint32_t p = (uint32_t)(y * A.W + x);
        uint32_t seed = init_seed(A.seed + p + (uint32_t)A.W * (uint32_t)A.H * (A.frame_index + f));
        float jx = 0.0f, jy = 0.0f;
        if (A.flags & kAA) { jx = random_float(seed); jy = random_float(seed); }           // :61
        const Ray r1 = primary_ray(S, (float)x, (float)y, A.W, A.H);
        B.seed[i] = seed;
        B.jit[i] = make_float2(jx, jy);
        B.ro[i] = make_float4(r1.O.x, r1.O.y, r1.O.z, 0.0f);
        B.rd[i] = make_float4(r1.D.x, r1.D.y, r1.D.z, 0.0f);
        B.info[i] = 0u;
        B.rinfo[i] = kRiFresh;
        B.pv[i] = 1u;
        B.s1[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);
        enq = true;
      } else {
        out[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);  // bounces == 0: Trace returns 0, t1 stays BVH_FAR
      }
    }
    // item i's home partition is i % kParts; a wave's 64 items cover every partition 8 times: one append per
    // (wave, partition), done by the lanes of that partition
    const uint32_t home = i % kParts;
    for (uint32_t p = 0; p < kParts; p++) {
      const bool mine = enq && home == p;
      if (!__ballot(mine)) continue;
      const uint32_t slot = wave_append(ctl_at(B.ctl, kSqRqTail + p), mine ? 1u : 0u);
      if (mine) {
        if (slot < B.cap_r) B.rq[(size_t)p * B.cap_r + slot] = (i << 3) | 4u;
        else atomicOr(ctl_at(B.ctl, kSqError), 1u);
      }
      const uint32_t nq = (uint32_t)__popcll(__ballot(mine));
      if (lane_id() == 0) {
        atomicAdd(ctl_at(B.ctl, kSqLive + p), nq);
        atomicAdd(ctl_at(B.ctl, kSqSegments + p), nq);
      }
    }
  }
}

// ---- NEE resolve of the item's last shading + stack unwind at a path end (resolve_item of prt_wave2.hip, no
// extensions); returns false when the path goes on (the result joined the stack)
__device__ __forceinline__ void stream_resolve(const TraceArgs& A, const StreamBufs& B, uint32_t item, uint32_t ri,
                                               uint32_t pvw, float4* __restrict__ out) {
  const uint32_t fl = A.flags;
  const uint32_t depth = ri & 0xFFu, path = (ri >> 8) & 1u, status = (ri >> 16) & 3u, kind = (ri >> 20) & 3u;
  const float4 ne = ld4(B.ne + item);
  V3 L = v3(ne.x, ne.y, ne.z);
  if (status == kStNeeEnd || status == kStNeeCont) {
    const float4 nb = ld4(B.nb + item);
    const uint32_t vis = (pvw >> 8) & 0xFu;
    V3 f[4];
    const uint32_t nr = kind == 0 ? 4u : 1u;
    for (uint32_t k = 0; k < 4; k++) {
      if (k < nr) {
        const float4 fk = ld4(B.nf + 4 * (size_t)item + k);
        f[k] = v3(fk.x, fk.y, fk.z);
      } else {
        f[k] = v3(0.0f, 0.0f, 0.0f);
      }
    }
    const V3 result = nee_resolve((int)kind, vis, L, v3(nb.x, nb.y, nb.z), f, fl);
    if (status == kStNeeCont) {  // the path goes on: result joins the stack
      B.R[(size_t)depth * B.n + item] = make_float4(result.x, result.y, result.z, 0.0f);
      return;
    }
    L = result;
  }
  for (int k = (int)depth - 1; k >= 0; k--) {                                              // result + Trace(..) * throughput
    const float4 Rk = ld4(B.R + (size_t)k * B.n + item), Tk = ld4(B.T + (size_t)k * B.n + item);
    L = v3(Rk.x, Rk.y, Rk.z) + L * v3(Tk.x, Tk.y, Tk.z);
  }
  const float4 s1 = ld4(B.s1 + item);
  if (path == 0 && (fl & kAA)) {  // path 2 follows; keep path 1's radiance
    B.s1[item] = make_float4(L.x, L.y, L.z, s1.w);
  } else {
    V3 res = (fl & kAA) ? 0.5f * (v3(s1.x, s1.y, s1.z) + L) : L;                           // :65
    if (fl & kGamma) res = v3(sqrtf(res.x), sqrtf(res.y), sqrtf(res.z));                  // :73-79
    out[item] = make_float4(res.x, res.y, res.z, s1.w);
  }
}

// ---- shading of the closest hit the item's last queued ray got (k_miss2 + k_shade2 of prt_wave2.hip for one item, no
// extensions).  Returns the rays to queue: shadow rays 0..nr-1 in bits 0-3, the next closest ray in bit 4; 0 when
// nothing is in flight (a miss that ends the path: the item's next visit resolves it at once)
__device__ __forceinline__ uint32_t stream_shade(const SceneDev& S, const TraceArgs& A, const TileMap& M,
                                                 const StreamBufs& B, uint32_t item) {
  const uint32_t fl = A.flags;
  const uint32_t info = ld1(B.info + item);
  const float4 hh = ld4(B.hit + item);
  const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u;
  if ((info & 0x1FFu) == 0) B.s1[item].w = hh.x;                                               // r1.hit.t
  uint32_t status = kStMiss, nr = 0;
  int kind = 0;
  bool next = false;
  if (hh.x >= kFar) {  // miss (:159): sky radiance or black ends the path
    V3 L = v3(0.0f, 0.0f, 0.0f);
    if (fl & kSkybox) {
      const float4 d = ld4(B.rd + item);
      L = sample_sky(S, v3(d.x, d.y, d.z));
    }
    B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
  } else {
    uint32_t seed = ld1(B.seed + item);
    kind = nee_kind(fl, seed);                                                                 // :198-214
    nr = (uint32_t)nee_rays(kind);
    const float4 o = ld4(B.ro + item), d = ld4(B.rd + item);
    const V3 D = v3(d.x, d.y, d.z);
    const uint32_t pk = __float_as_uint(hh.w);
    const V3 I = v3(o.x, o.y, o.z) + hh.x * D;                                                 // tiny_bvh.h:586
    const V3 V = -D;
    const HitAttr ha = hit_attributes(S, hit_inst(S, pk), hit_prim(S, pk), hh.y, hh.z, (fl & kNormalMap) != 0);
    const V3 e = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * ha.m.emis;                    // :196
    B.ne[item] = make_float4(e.x, e.y, e.z, 0.0f);
    float4* sho = B.sho + 4 * (size_t)item;
    float4* shd = B.shd + 4 * (size_t)item;
    float4* nf = B.nf + 4 * (size_t)item;
    const V3 brdf = nee_lights(S, fl, kind, I, V, ha.N, ha.m, seed, [&](int k, const Ray& sr, float tmax, V3 fk) {
      sho[k] = make_float4(sr.O.x, sr.O.y, sr.O.z, tmax);
      shd[k] = make_float4(sr.D.x, sr.D.y, sr.D.z, 0.0f);
      nf[k] = make_float4(fk.x, fk.y, fk.z, 0.0f);
    });
    B.nb[item] = make_float4(brdf.x, brdf.y, brdf.z, 0.0f);
    status = kStNeeEnd;
    if ((int)depth != A.bounces - 1) {                                                         // :329
      V3 dir, thr;
      if (sample_bounce(ha.m, V, ha.N, seed, dir, thr)) {                                      // :376-399
        status = kStNeeCont;
        B.T[(size_t)depth * B.n + item] = make_float4(thr.x, thr.y, thr.z, 0.0f);
        const Ray nr2 = make_ray(I + dir * kEpsilon, dir);                                     // :404
        B.ro[item] = make_float4(nr2.O.x, nr2.O.y, nr2.O.z, 0.0f);
        B.rd[item] = make_float4(nr2.D.x, nr2.D.y, nr2.D.z, 0.0f);
        B.info[item] = (depth + 1u) | (path << 8);
        next = true;
      }
    }
    B.seed[item] = seed;
  }
  if (status != kStNeeCont && path == 0 && (fl & kAA)) {  // path 1 ends: path 2's primary ray (jitter drawn at :61)
    const uint32_t r = (B.base + item) % M.items;
    int32_t x, y;
    item_pixel(M, r, x, y);
    const float2 j = ld2(B.jit + item);
    const Ray r2 = primary_ray(S, (float)x + j.x, (float)y + j.y, A.W, A.H);
    B.ro[item] = make_float4(r2.O.x, r2.O.y, r2.O.z, 0.0f);
    B.rd[item] = make_float4(r2.D.x, r2.D.y, r2.D.z, 0.0f);
    B.info[item] = 1u << 8;
    next = true;
  }
  B.rinfo[item] = depth | (path << 8) | (status << 16) | ((uint32_t)kind << 20) | (next ? kRiQueued : 0u);
  const uint32_t rays = ((1u << nr) - 1u) | (next ? 0x10u : 0u);
  B.pv[item] = (uint32_t)__popc(rays);
  return rays;
}

// ---- the persistent launch
template <bool TLAS>
__global__ void __launch_bounds__(64, kStreamWaves) k_stream(SceneDev S, TraceArgs A, TileMap M, StreamBufs B,
                                                            float4* __restrict__ out) {
  __shared__ uint32_t lds_stack[2 * kStreamStack * 64];
  const uint32_t part = xcc_id();
  uint32_t* ctl = B.ctl;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  uint32_t rtk = kNoTk, stk = kNoTk;  // tickets held across phases (ray queue, shade queue)
  uint32_t n_seg = 0, n_sh = 0;       // rays this wave queued (wave-uniform, stats)
  uint32_t idle_rounds = 0;           // consecutive rounds without work (sleep back-off)
  while (true) {
    bool worked = false;
    // ------------------------------------------------------------ traversal phase
    {
      bool have = false;
      // Publication of finished rays, one step per traversal iteration (tick, wave-uniform):
      //   closest ray: hit stored (cl_item) -> next tick: drain, pending-word atomic (c_item, c_old) -> next tick: last?
      //   shadow ray:  pending-word atomic with its visibility bit at once (s_item, s_old) -> next tick: last?
      // so the atomics' latency overlaps an iteration and one drain serves every lane of the wave
      uint32_t cl_item = kNoTk, c_item = kNoTk, c_old = 0, s_item = kNoTk, s_old = 0;
      auto publish = [&]() {  // wave-uniform
        const uint32_t p0 = (c_item != kNoTk && (c_old & 0xFFu) == 1u) ? c_item : kNoTk;
        const uint32_t p1 = (s_item != kNoTk && (s_old & 0xFFu) == 1u) ? s_item : kNoTk;
        c_item = s_item = kNoTk;
        const uint32_t np = (p0 != kNoTk ? 1u : 0u) + (p1 != kNoTk ? 1u : 0u);
        if (__ballot(np != 0u)) {
          const uint32_t slot = wave_append(ctl_at(ctl, kSqSqTail + part), np);
          uint32_t j = 0;
          for (uint32_t q : {p0, p1}) {
            if (q == kNoTk) continue;
            if (slot + j < B.cap_s) st_rlx(B.sq + (size_t)part * B.cap_s + slot + j, q);
            else atomicOr(ctl_at(ctl, kSqError), 1u);
            j++;
          }
        }
        if (__ballot(cl_item != kNoTk)) {
          drain_stores();  // the hit records are out before the pending words say so
          if (cl_item != kNoTk) {
            c_old = atomicAdd(&B.pv[cl_item], 0xFFFFFFFFu);
            c_item = cl_item;
            cl_item = kNoTk;
          }
        }
      };
      trav8_persistent_t<2, kStreamStack, 32, 32, TLAS, false, true>(
          S, lds_stack + threadIdx.x,
          [&](uint32_t*, uint32_t) -> uint32_t {  // claim tickets for the idle lanes without one
            const uint64_t free_m = __ballot(rtk == kNoTk);
            uint32_t first = 0;
            const uint32_t got = free_m ? claim(ctl, kSqRqTail, kSqRqHead, part, (uint32_t)__popcll(free_m), first) : 0u;
            const uint32_t rank = (uint32_t)__popcll(free_m & ((1ull << lane_id()) - 1ull));
            if (rtk == kNoTk && rank < got) rtk = first + rank;
            return got;
          },
          [&](uint32_t e, V3& O, V3& D, float& tmax, bool& any) -> uint32_t {  // queue entry -> world ray
            acquire();
            const uint32_t item = e >> 3, k = e & 7u;
            float4 o, d;
            if (k == 4u) {
              o = ld4(B.ro + item);
              d = ld4(B.rd + item);
              tmax = kFar;
              any = false;
            } else {
              o = ld4(B.sho + 4 * (size_t)item + k);
              d = ld4(B.shd + 4 * (size_t)item + k);
              tmax = o.w;
              any = true;
            }
            O = v3(o.x, o.y, o.z);
            D = v3(d.x, d.y, d.z);
            have = true;
            return e;
          },
          [&](uint32_t e, bool any, V3& O, V3& D) {
            const uint32_t item = e >> 3, k = e & 7u;
            const float4 o = ld4(any ? B.sho + 4 * (size_t)item + k : B.ro + item);
            const float4 d = ld4(any ? B.shd + 4 * (size_t)item + k : B.rd + item);
            O = v3(o.x, o.y, o.z);
            D = v3(d.x, d.y, d.z);
          },
          [&](uint32_t e, const Hit& hit, bool any, bool occluded) {
            const uint32_t item = e >> 3, k = e & 7u;
            if (any) {
              s_old = atomicAdd(&B.pv[item], (occluded ? 0u : (1u << (8 + k))) - 1u);
              s_item = item;
            } else {
              B.hit[item] = make_float4(hit.t, hit.u, hit.v, __uint_as_float(pack_hit(S, hit.prim, hit.inst)));
              cl_item = item;
            }
          },
          [&](uint32_t, bool) { publish(); }, nullptr,
          [&]() -> uint32_t {  // this lane's ticketed entry, once written
            if (rtk == kNoTk) return kStreamEmpty;
            const uint32_t v = take(B.rq, B.cap_r, rtk);
            if (v != kStreamEmpty) rtk = kNoTk;
            return v;
          });
      publish();  // settle the last iteration's finishes: closest atomics issued ...
      publish();  // ... and their results queued
      worked |= __ballot(have) != 0;
    }
    // ------------------------------------------------------------ shading phase: one item per lane
    {
      const uint64_t free_m = __ballot(stk == kNoTk);
      if (free_m) {
        uint32_t first = 0;
        const uint32_t got = claim(ctl, kSqSqTail, kSqSqHead, part, (uint32_t)__popcll(free_m), first);
        const uint32_t rank = (uint32_t)__popcll(free_m & ((1ull << lane_id()) - 1ull));
        if (stk == kNoTk && rank < got) stk = first + rank;
      }
      uint32_t item = kNoTk;
      if (stk != kNoTk) {
        item = take(B.sq, B.cap_s, stk);
        if (item != kStreamEmpty) stk = kNoTk;
        else item = kNoTk;
      }
      if (__ballot(item != kNoTk)) {
        worked = true;
        // resolve what the item's last visit left in flight, then shade its new hit (two separate passes over
        // the wave's items, so their registers are not live together)
        uint32_t ri = 0;
        acquire();
        if (item != kNoTk) {
          ri = ld1(B.rinfo + item);
          if (!(ri & kRiFresh)) stream_resolve(A, B, item, ri, ld1(B.pv + item), out);
        }
        const bool go = item != kNoTk && (ri & (kRiQueued | kRiFresh));
        const bool done = item != kNoTk && !go;
        uint32_t rays = 0;
        if (go) rays = stream_shade(S, A, M, B, item);
        const bool again = go && rays == 0u;  // nothing in flight: the next visit resolves it (pv = 0: no vis bits)
        drain_stores();  // the item's state is out before its rays (or itself) are queued
        const uint32_t nrays = (uint32_t)__popc(rays);
        const uint32_t slot = wave_append(ctl_at(ctl, kSqRqTail + part), nrays);
        uint32_t j = 0;
        for (uint32_t k = 0; k < 5; k++) {
          if (rays & (1u << k)) {
            if (slot + j < B.cap_r) st_rlx(B.rq + (size_t)part * B.cap_r + slot + j, (item << 3) | k);
            else atomicOr(ctl_at(ctl, kSqError), 1u);
            j++;
          }
        }
        if (__ballot(again)) {
          const uint32_t s2 = wave_append(ctl_at(ctl, kSqSqTail + part), again ? 1u : 0u);
          if (again) {
            if (s2 < B.cap_s) st_rlx(B.sq + (size_t)part * B.cap_s + s2, item);
            else atomicOr(ctl_at(ctl, kSqError), 1u);
          }
        }
        n_seg += (uint32_t)__popcll(__ballot((rays >> 4) & 1u));
        n_sh += nrays_w(rays);
        const uint32_t nd = (uint32_t)__popcll(__ballot(done));
        if (lane_id() == 0 && nd) atomicSub(ctl_at(ctl, kSqLive + part), nd);
      }
    }
    if (__builtin_amdgcn_s_memrealtime() - t_start > kStreamLimit) {  // never hang the GPU: fail the call
      if (lane_id() == 0) atomicOr(ctl_at(ctl, kSqError), 2u);
      break;
    }
    if (worked) {
      idle_rounds = 0;
    } else {  // this XCD's items all finished (or the call failed)?
      uint32_t live = 0, err = 0;
      if (lane_id() == 0) {
        live = ld_ctl(ctl_at(ctl, kSqLive + part));
        err = ld_ctl(ctl_at(ctl, kSqError));
      }
      if (__shfl((int)live, 0, 64) == 0 || __shfl((int)err, 0, 64) != 0) break;
      // back off: idle waves polling the queue counters slow the atomics of the waves that have work
      if (idle_rounds < 2) __builtin_amdgcn_s_sleep(8);
      else if (idle_rounds < 8) __builtin_amdgcn_s_sleep(32);
      else __builtin_amdgcn_s_sleep(127);
      idle_rounds++;
    }
  }
  if (lane_id() == 0) {  // ray counts
    if (n_seg) atomicAdd(ctl_at(ctl, kSqSegments + part), n_seg);
    if (n_sh) atomicAdd(ctl_at(ctl, kSqShadow + part), n_sh);
  }
}

hipError_t launch_stream(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M, const StreamBufs& B,
                         float4* out) {
  if (B.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_stream_init, dim3(256u * 4u), dim3(kBlock), 0, c.stream, S, A, M, B, out);
  if (S.tlas)
    hipLaunchKernelGGL(k_stream<true>, dim3(kStreamBlocks), dim3(64), 0, c.stream, S, A, M, B, out);
  else
    hipLaunchKernelGGL(k_stream<false>, dim3(kStreamBlocks), dim3(64), 0, c.stream, S, A, M, B, out);
  return hipGetLastError();
}

}  // namespace prt
