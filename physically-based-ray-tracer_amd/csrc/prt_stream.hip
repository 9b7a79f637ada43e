// prt_stream.hip -- streaming path engine (PRT_PIPELINE=stream) for gfx950.
//
// The merged pipeline (prt_wave2.hip) runs every bounce as its own launches, so each bounce waits for
// the slowest ray of the one before: on 1/8 of a 1080p frame per GPU those launch tails are about half
// the frame (scripts/rank_time.py).  Here ONE persistent launch carries the whole frame batch and every
// wave switches between two roles:
//   trace   persistent-lane Node8 traversal (prt_persist.h) of ray ids taken from the ray queue; the ray
//           that brings its item's in-flight count to zero hands the item to the shade queue
//   shade   up to 64 items from the shade queue: first the NEE resolve of the item's previous bounce
//           (its shadow rays are done), then its current hit -- sky / debug colour / BRDF shading with
//           the NEE set-up and the sampled bounce or the AA path-2 primary ray -- whose rays go to the
//           ray queue
// so an item's next bounce starts as soon as its own rays are done.  Per item the work and every random
// draw happen in the merged pipeline's order (resolve(i-1) then shade(i), the same WaveBufs state), so
// the image is bit-identical to it.
//
// Placement and visibility (MI355X_MICROARCH.md, inter-workgroup visibility).  Items are dealt to XCD
// parts by 64-item chunk and every ray and shading task of an item runs on a wave of its part's XCD
// (HW_REG_XCC_ID, mapped by a census at context creation), so each hand-off stays inside one L2:
// producers store plainly (the vector L1 is write-through), drain with s_waitcnt vmcnt(0), then store
// the tagged 8-byte granule that publishes the work; consumers poll the granule with an sc1 load and
// read every handed-off byte with sc1 loads (L1 bypassed, L2 served).  In-flight counts, queue counters,
// the live counts and the abort word are touched by agent atomics and sc1 loads / stores only.  Queues
// are linear (written once per launch) and granules carry the launch serial, so the granule arrays are
// never cleared.  A watchdog (s_memrealtime) and an abort word bound every wait.
#include "prt_launch.h"
#include "prt_path.h"
#include "prt_persist.h"
#include "prt_queue.h"
#include "prt_bounce.h"

namespace prt {

namespace {

using u64 = unsigned long long;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

constexpr uint32_t kShadowBit = 0x80000000u;
constexpr uint32_t kNone = 0xFFFFFFFFu;
enum : uint32_t { kErrTimeout = 1, kErrOverflow = 2, kErrState = 3 };

__device__ __forceinline__ uint32_t ld1(const uint32_t* p) {
  return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld1(const u64* p) {
  return __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// 16-B sc1 load at a byte offset (< 4 GiB, checked on the host) of a uniform base
__device__ __forceinline__ float4 ld4(const void* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
  const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);  // aux 16 = sc1
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ float4 ld4(const float4* a, uint32_t i) { return ld4((const void*)a, i * 16u); }
// the streaming engine's loads of handed-off item state (sc1: L1 bypassed, L2 served)
struct Sc1Loads {
  static __device__ __forceinline__ uint32_t u32(const uint32_t* p) { return ld1(p); }
  static __device__ __forceinline__ float4 f4(const float4* a, uint32_t i) { return ld4(a, i); }
};
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint64_t clock100() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// counters: which = 0 ray tail, 1 ray head, 2 shade tail, 3 shade head
__device__ __forceinline__ uint32_t* qctr(const StreamBufs& Q, uint32_t part, uint32_t which, uint32_t s) {
  return Q.ctr + ((part * 4u + which) * kSSub + s) * kCtrStride;
}
__device__ __forceinline__ uint32_t* live_ctr(const StreamBufs& Q, uint32_t part) {
  return Q.ctl + (2u + part) * kCtrStride;
}
__device__ __forceinline__ void raise_error(const StreamBufs& Q, uint32_t code) {
  atomicCAS(Q.ctl + 1, 0u, code);  // the first error is kept
  st1(Q.ctl, 1u);
}

// one sc1 load per lane: lanes 0..31 the part's queue counters, 32 the abort word, 33 the live count
__device__ __forceinline__ uint32_t read_state(const StreamBufs& Q, uint32_t part) {
  const uint32_t l = lane_id();
  const uint32_t* p = l < 4u * kSSub ? Q.ctr + (part * 4u * kSSub + l) * kCtrStride
                                     : (l == 32u ? Q.ctl : live_ctr(Q, part));
  return l < 34u ? ld1(p) : 0u;
}
// entries published or reserved in queue q (0 ray, 1 shade) summed over the sub-queues
__device__ __forceinline__ uint32_t backlog(uint32_t v, uint32_t q) {
  const uint32_t s = lane_id() & (kSSub - 1u);
  const uint32_t t = __shfl(v, (int)(16u * q + s)), h = __shfl(v, (int)(16u * q + 8u + s));
  uint32_t a = (lane_id() < kSSub && t > h) ? t - h : 0u;
  a += __shfl_xor(a, 1);
  a += __shfl_xor(a, 2);
  a += __shfl_xor(a, 4);
  return __shfl(a, 0);
}

// wave-uniform claim of up to `want` consecutive entries of queue q in the part: the sub-queue with the
// most entries in the counter snapshot v (ties: round-robin), its head advanced by CAS up to the tail
// (retried while entries remain).  Returns the count; *slot = index of the first granule.
__device__ __forceinline__ uint32_t claim(const StreamBufs& Q, uint32_t part, uint32_t q, uint32_t want, uint32_t v,
                                          uint32_t& rot, uint32_t* slot) {
  const uint32_t l = lane_id(), s = l & (kSSub - 1u);
  const uint32_t t = __shfl(v, (int)(16u * q + s)), h = __shfl(v, (int)(16u * q + 8u + s));
  const uint32_t av = (l < kSSub && t > h) ? t - h : 0u;
  uint32_t best = av;
  for (int o = 1; o < (int)kSSub; o <<= 1) best = max(best, (uint32_t)__shfl_xor(best, o));
  best = __shfl(best, 0);
  if (best == 0) return 0;
  const uint32_t m = (uint32_t)__ballot(l < kSSub && av >= min(best, want)) & 0xFFu;
  const uint32_t r = rot & 7u;
  rot++;
  const uint32_t rm = ((m >> r) | (m << (8u - r))) & 0xFFu;
  const uint32_t sub = (__builtin_ctz(rm) + r) & 7u;
  uint32_t got = 0, base = 0;
  uint32_t hs = __shfl(h, (int)sub), ts = __shfl(t, (int)sub);
  if (l == 0) {
    uint32_t* hp = qctr(Q, part, 2u * q + 1u, sub);
    for (int tries = 0; tries < 64 && ts > hs; tries++) {
      const uint32_t k = min(want, ts - hs);
      const uint32_t old = atomicCAS(hp, hs, hs + k);
      if (old == hs) { got = k; base = hs; break; }
      hs = old;
      if (ts <= hs) ts = ld1(qctr(Q, part, 2u * q, sub));
    }
  }
  got = __shfl(got, 0);
  base = __shfl(base, 0);
  *slot = (part * kSSub + sub) * (q ? Q.hcap : Q.rcap) + base;
  return got;
}

// wave-uniform append: lane i contributes cnt_i (0..7) ids id(k), k < cnt_i; one atomic per wave
template <class Id>
__device__ __forceinline__ void push(const StreamBufs& Q, uint32_t part, uint32_t q, uint32_t cnt, uint32_t& rot, Id id) {
  const uint64_t b1 = __ballot(cnt & 1u), b2 = __ballot(cnt & 2u), b4 = __ballot(cnt & 4u);
  const uint32_t tot = (uint32_t)__popcll(b1) + 2u * (uint32_t)__popcll(b2) + 4u * (uint32_t)__popcll(b4);
  if (tot == 0) return;
  const uint64_t lt = (1ull << lane_id()) - 1ull;
  const uint32_t before = (uint32_t)__popcll(b1 & lt) + 2u * (uint32_t)__popcll(b2 & lt) + 4u * (uint32_t)__popcll(b4 & lt);
  const uint32_t sub = rot & 7u;
  rot++;
  const uint32_t cap = q ? Q.hcap : Q.rcap;
  uint32_t base = 0;
  if (lane_id() == 0) base = atomicAdd(qctr(Q, part, 2u * q, sub), tot);
  base = __shfl(base, 0);
  if (base + tot > cap) {
    if (lane_id() == 0) raise_error(Q, kErrOverflow);
    return;
  }
  u64* g = (q ? Q.hq : Q.rq) + (size_t)(part * kSSub + sub) * cap + base + before;
  const u64 tag = (u64)Q.serial << 32;
  for (uint32_t k = 0; k < cnt; k++) g[k] = tag | id(k);
}

// the published id of granule g (polls until its tag is this launch's); kNone on abort / watchdog
__device__ __forceinline__ uint32_t wait_granule(const StreamBufs& Q, const u64* g, uint64_t deadline) {
  for (uint32_t spin = 0;; spin++) {
    const u64 x = ld1(g);
    if ((uint32_t)(x >> 32) == Q.serial) return (uint32_t)x;
    if ((spin & 31u) == 31u && (ld1(Q.ctl) != 0 || clock100() > deadline)) {
      raise_error(Q, kErrTimeout);
      return kNone;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

template <bool HALF, int REFILL, int STACK, int WAVES>
__global__ void __launch_bounds__(64, WAVES) k_stream(SceneDev S, TraceArgs A, TileMap M, WaveBufs B, StreamBufs Q,
                                                      float4* __restrict__ out) {
  __shared__ uint32_t lds_stack[2 * STACK * 64];
  const uint32_t part = (Q.xcc_part >> (4u * xcc_id())) & 0xFu;
  if (part >= Q.nparts) return;
  const uint64_t t_start = clock100();
  const uint64_t deadline = t_start + (uint64_t)Q.budget_ms * 100000ull;
  // shading backlog at which this wave stops taking rays: spread over 64..2048 items so that the share of
  // waves turning to shading follows the backlog
  const uint32_t shade_thr = 64u * (1u + ((blockIdx.x >> 3) & 31u));
  uint8_t* vis8 = reinterpret_cast<uint8_t*>(B.vis);
  uint32_t rot = blockIdx.x;
  uint32_t nseg = 0, nsh = 0;
  uint64_t t_shade = 0, t_trace = 0, n_batch = 0, n_items = 0;
  uint32_t cdone = kNone;  // item of the ray this lane finished whose in-flight count is not yet decremented
  // publish finished rays: one drain for the wave's hit / visibility stores, the in-flight decrements, and
  // the items whose count reached zero into the shade queue
  auto complete = [&]() {
    drain();
    uint32_t ready = kNone;
    if (cdone != kNone && atomicSub(Q.pend + cdone, 1u) == 1u) ready = cdone;
    cdone = kNone;
    const bool v = ready != kNone;
    push(Q, part, 1u, v ? 1u : 0u, rot, [&](uint32_t) { return ready; });
  };
  for (;;) {
    const uint32_t v = read_state(Q, part);
    if (__shfl(v, 32) != 0u || __shfl(v, 33) == 0u) break;
    const uint32_t hq = backlog(v, 1u);
    uint32_t slot = 0, hgot = 0;
    if (hq >= 64u || (hq && backlog(v, 0u) == 0u)) hgot = claim(Q, part, 1u, 64u, v, rot, &slot);
    if (hgot) {  // ---- shade role
      const uint64_t t0 = clock100();
      const uint32_t l = lane_id();
      uint32_t item = kNone;
      if (l < hgot) item = wait_granule(Q, Q.hq + slot + l, deadline);
      bool done = false;
      uint32_t hasC = 0, nS = 0;
      if (item != kNone) {
        shade_item<Sc1Loads>(S, A, M, B, item, out, false, done, hasC, nS);
        if (!done && hasC + nS == 0) raise_error(Q, kErrState);
        if (hasC + nS) st1(Q.pend + item, hasC + nS);  // in-flight count before the rays are published
      }
      drain();
      push(Q, part, 0u, hasC + nS, rot, [&](uint32_t k) {
        return (hasC && k == 0) ? item : (kShadowBit | (4u * item + (k - hasC)));
      });
      const uint32_t nd = (uint32_t)__popcll(__ballot(done));
      if (nd && l == 0) atomicSub(live_ctr(Q, part), nd);
      t_shade += clock100() - t0;
      n_batch++;
      n_items += hgot;
      continue;
    }
    // ---- trace role
    const uint64_t t0 = clock100();
    bool traced = false;
    trav8_persistent_t<2, HALF, STACK, REFILL>(
        S, lds_stack + threadIdx.x,
        [&](uint32_t* base, uint32_t want) -> uint32_t {
          const uint32_t v2 = read_state(Q, part);
          if (__shfl(v2, 32) != 0u || backlog(v2, 1u) >= shade_thr) return 0u;
          const uint32_t got = claim(Q, part, 0u, want, v2, rot, base);
          traced |= got != 0;
          return got;
        },
        [&](uint32_t g, V3& O, V3& D, float& tmax, bool& any) -> uint32_t {
          const uint32_t id = wait_granule(Q, Q.rq + g, deadline);
          float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
          if (id == kNone) {
            any = true;
          } else if (id & kShadowBit) {
            o = ld4(B.sho, id & ~kShadowBit);
            d = ld4(B.shd, id & ~kShadowBit);
            any = true;
          } else {
            o = ld4(B.ro, id);
            d = ld4(B.rd, id);
            o.w = kFar;
            any = false;
          }
          O = v3(o.x, o.y, o.z);
          D = v3(d.x, d.y, d.z);
          tmax = o.w;
          return id;
        },
        [&](uint32_t h, bool any, V3& O, V3& D) {
          float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f), d = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
          if (h != kNone) {
            o = any ? ld4(B.sho, h & ~kShadowBit) : ld4(B.ro, h);
            d = any ? ld4(B.shd, h & ~kShadowBit) : ld4(B.rd, h);
          }
          O = v3(o.x, o.y, o.z);
          D = v3(d.x, d.y, d.z);
        },
        [&](uint32_t h, const Hit& hit, bool any, bool occluded) {
          if (h == kNone) return;
          if (any) {
            const uint32_t k = h & ~kShadowBit;
            if (!occluded) vis8[k] = 1;
            cdone = k >> 2;
            nsh++;
          } else {
            B.hit[h] = make_float4(hit.t, hit.u, hit.v, __uint_as_float(pack_hit(hit.prim, hit.inst)));
            cdone = h;
            nseg++;
          }
        },
        // a lane holds at most one finished ray: it stays idle until the next refill, so publishing right
        // before each refill (and in batches of 16 once no refill is coming) keeps one drain per refill
        [&](uint32_t idle, bool drained) {
          const uint64_t pm = __ballot(cdone != kNone);
          if (pm && (drained ? __popcll(pm) >= 16 : idle >= (uint32_t)REFILL)) complete();
        });
    if (__ballot(cdone != kNone)) complete();
    t_trace += clock100() - t0;
    if (!traced) {
      if (clock100() > deadline) {
        if (lane_id() == 0) raise_error(Q, kErrTimeout);
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
  }
  const uint32_t a = wave_sum(nseg), b = wave_sum(nsh);
  if (lane_id() == 0) {
    if (a) atomicAdd(Q.stat, (u64)a);
    if (b) atomicAdd(Q.stat + 1, (u64)b);
    atomicAdd(Q.stat + 2, (u64)t_shade);
    atomicAdd(Q.stat + 3, (u64)t_trace);
    atomicAdd(Q.stat + 4, (u64)(clock100() - t_start));
    atomicAdd(Q.stat + 5, n_batch);
    atomicAdd(Q.stat + 6, n_items);
  }
}

// init: seeds, AA jitter, primary ray r1 of every item; each wave's 64 items (one part) into its ray queue
__global__ void __launch_bounds__(kBlock) k_stream_init(SceneDev S, TraceArgs A, TileMap M, WaveBufs B, StreamBufs Q,
                                                        float4* __restrict__ out) {
  for (uint32_t c = blockIdx.x; c * kBlock < B.n; c += gridDim.x) {
    const uint32_t i = c * kBlock + threadIdx.x;
    bool enq = false;
    if (i < B.n) {
      const uint32_t f = i / M.items, r = i % M.items;
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
        B.info[i] = kHitPending;
        B.rinfo[i] = 0u;
        B.s1[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);
        st1(Q.pend + i, 1u);
        enq = true;
      } else if (i < B.n) {
        out[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);  // bounces == 0: Trace returns 0, t1 stays BVH_FAR
      }
    }
    const uint64_t m = __ballot(enq);
    if (m) {
      const uint32_t chunk = (c * kBlock + (threadIdx.x & ~63u)) >> 6;
      const uint32_t part = chunk % Q.nparts, sub = (chunk / Q.nparts) % kSSub;
      const uint32_t cnt = (uint32_t)__popcll(m);
      uint32_t base = 0;
      if (lane_id() == 0) {
        base = atomicAdd(qctr(Q, part, 0u, sub), cnt);
        atomicAdd(live_ctr(Q, part), cnt);
      }
      base = __shfl(base, 0);
      if (base + cnt > Q.rcap) {
        if (lane_id() == 0) raise_error(Q, kErrOverflow);
      } else if (enq) {
        const uint32_t rank = (uint32_t)__popcll(m & ((1ull << lane_id()) - 1ull));
        st1(Q.rq + (size_t)(part * kSSub + sub) * Q.rcap + base + rank, ((u64)Q.serial << 32) | i);
      }
    }
  }
}

__global__ void k_xcc_census(uint32_t* mask) {
  if (threadIdx.x == 0) atomicOr(mask, 1u << xcc_id());
}

template <int REFILL, int STACK, int WAVES>
void launch_s(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M, const WaveBufs& B,
              const StreamBufs& Q, float4* out, uint32_t cus) {
  const dim3 grid(cus * 4u * WAVES);
  if (c.layout == 9)
    hipLaunchKernelGGL((k_stream<true, REFILL, STACK, WAVES>), grid, dim3(64), 0, c.stream, S, A, M, B, Q, out);
  else
    hipLaunchKernelGGL((k_stream<false, REFILL, STACK, WAVES>), grid, dim3(64), 0, c.stream, S, A, M, B, Q, out);
}

}  // namespace

hipError_t launch_xcc_census(hipStream_t s, uint32_t* dev_mask) {
  hipLaunchKernelGGL(k_xcc_census, dim3(8192), dim3(64), 0, s, dev_mask);
  return hipGetLastError();
}

hipError_t launch_stream(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                         const WaveBufs& B, const StreamBufs& Q, float4* out) {
  if (B.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_stream_init, dim3(256u * 4u), dim3(kBlock), 0, c.stream, S, A, M, B, Q, out);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (Q.waves == 4) launch_s<32, 16, 4>(c, S, A, M, B, Q, out, (uint32_t)cus);
  else launch_s<32, 12, 5>(c, S, A, M, B, Q, out, (uint32_t)cus);
  return hipGetLastError();
}

}  // namespace prt
