// prt_launch.h -- host-side launchers implemented in prt_render.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "prt_kernels.h"
#include "prt_post.h"
#include "prt_traverse8.h"

namespace prt {

struct Counters {
  unsigned long long segments, shadow;
};
struct HitOut {
  float t, u, v;
  uint32_t prim, inst;
};
struct LaunchCfg {
  hipStream_t stream;
  int occ;     // persistent traversal waves/SIMD: 7 / 6 / 5 / 4 (9 / 11 / 14 / 18 LDS stack groups)
  uint32_t groups = 1;  // grid divisor: every wavefront grid is 1/groups of the resident blocks (frames in flight:
                        // the chains' persistent launches co-reside on the SIMDs, prt_api.cpp enqueue_render)
};

// wavefront pipeline buffers (SoA over n work items; R/T hold (bounces-1) x n entries)
constexpr uint32_t kNSub = 32;       // sub-queues per queue (one append counter each)
constexpr uint32_t kCtrStride = 32;  // words between counters (each on its own 128-B line)
struct WaveBufs {
  uint32_t n;       // items of this call
  uint32_t base;    // first item of the state arrays within the call (0)
  uint32_t qcap;    // capacity of one path sub-queue  (multiple of 256)
  uint32_t scap;    // capacity of one shadow sub-queue (4 x qcap)
  uint32_t* seed;
  uint32_t* info;   // depth | path << 8 | status << 16 | nee kind << 20
  uint32_t* rinfo;  // merged pipeline: what k_resolve2 finishes (depth | path << 8 | status << 16 | kind << 20)
  float4* ro;
  float4* rd;
  float4* R;
  float4* T;
  float4* s1;       // path-1 radiance, w = r1.hit.t
  float2* jit;
  float4* hit;      // t, u, v, bits(prim | inst << 26)
  float4* ne;       // emissive (or the path's end value)
  float4* nb;       // NEE BRDF value
  float4* nk;       // NEE factors the shadow rays' contributions are rebuilt from (prt_path.h nee_lights)
  uint32_t* vis;    // 4 visibility bytes per item
  uint32_t* q0;
  uint32_t* q1;
  uint32_t* shq;    // shadow queue: light << 29 | visibility index (prt_wave2.hip shadow_of)
  float4* hp;       // the hit point I of the item's last shading (its shadow rays' origin before the offset)
  uint32_t* ctr;    // [iteration][path|shadow][sub-queue] counters, kCtrStride apart
  // extensions (area light / dielectric instances; merged pipeline only): vis holds 5 x n bytes, the area
  // light's shadow ray writes byte 4 * n + item
  float4* na;       // area-light NEE contribution before visibility
  uint32_t* dst;    // dielectric DFS state: bits 0-7 dielectric level, 8-15 refraction started,
                    // 16-23 reflected radiance stored (in T[level]), 24-31 no refraction (k <= 0)
  float4* dro;      // per level: refraction ray origin, fresnel
  float4* drd;      // per level: refraction ray direction
  float4* ao;       // the area light's shadow ray per item: origin, tmax (its NEE sample is random: stored whole)
  float4* ad;       // ... direction
  unsigned long long* tl;  // PRT_DEBUG_QUEUES: [launch][wave] {start, first empty fetch, exit, -}
  int32_t coop_tail;       // cooperative traversal tail (prt_persist.h)
  int32_t merge;           // path-2 merge (prt_wave2.hip): the AA path-2 primaries traced with path 1's, and
                           // each path's NEE record / (result, throughput) stack in its own slot (slot p at p * n)
  float4* ro2;             // merge: the path-2 primary ray (k_wave_init), traced by k_trace2(0) ...
  float4* rd2;
  float4* hit2;            // ... into hit2; shaded by k_shade2 right after path 1 ends
};
constexpr uint32_t kParts = 8;  // XCD parts of a traversal launch's live range, one fetch counter each (prt_queue.h)
constexpr int kMaxIters = 128;  // wavefront iterations per call: bounces <= 64 (AA) / 6 with dielectrics (AA)
#ifdef PRT_LANE_STATS
void lane_stats_dump();  // diagnostic build: prints and clears the traversal lane counters (prt_wave2.hip)
#endif
// wavefront iterations of one call: one per path segment, paths x bounces; with dielectric instances a path
// is a binary tree walked depth first (one segment per iteration), at most 2^bounces - 1 segments per path
inline uint32_t wave_iters(bool dielectric, int bounces, uint32_t flags, bool merge = false) {
  const uint32_t paths = (flags & 1u) ? 2u : 1u;  // PRT_FLAG_AA: two camera paths per reference frame
  // merged: path 2's first segment is shaded in the iteration path 1 ends in (its primary hit traced up front)
  if (merge && paths == 2 && bounces > 0) return 2u * (uint32_t)bounces - 1u;
  if (!dielectric) return paths * (uint32_t)bounces;
  return bounces > 8 ? 0xFFFFFFFFu : paths * ((1u << bounces) - 1u);  // dst holds 4 bits per level for 8 levels
}
constexpr int kTlWaves = 256 * 4 * 8;  // timeline records per traversal launch (max persistent grid)
struct WaveTimers {
  hipEvent_t ev[4 * (kMaxIters + 1)];
  uint32_t iters;
};

hipError_t launch_wave_init(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                            const WaveBufs& B, float4* out);
// merged pipeline (prt_wave2.hip): iteration `it` (0..iters) after launch_wave_init -- one traversal launch for
// P(it) closest + S(it-1) any-hit, then resolve / miss / shade
hipError_t launch_wave2_iter(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                             const WaveBufs& B, float4* out, WaveTimers* tm, uint32_t it);
// zero na words at a and nb words at b (one dispatch)
hipError_t launch_clear2(const LaunchCfg& c, uint32_t* a, uint32_t na, uint32_t* b, uint32_t nb);
// acc_prev (nullable): the accumulator state before the last frame of the call (screen-pass input);
// totals (nullable): running ray totals, incremented by the queue counters ctr of the pass's `iters` iterations
hipError_t launch_accumulate(const LaunchCfg& c, const TileMap& M, int32_t frames, uint32_t flags, const float4* fr,
                             float4* acc, int32_t* nsamp, float* dist, float4* avg, uint32_t* rgb8, float4* tiles,
                             float4* acc_prev, const uint32_t* ctr, uint32_t iters, Counters* totals);
// post-processed RGB8 of the whole image (Core/Renderer.cpp:107-133)
hipError_t launch_postfx(const LaunchCfg& c, const PostDev& P, const float4* acc_new, const float4* acc_old,
                         const int32_t* nsamp, const float4* avg, uint32_t* rgb8);
hipError_t launch_untile(const LaunchCfg& c, int32_t W, int32_t H, int32_t ts, int32_t world, uint32_t per_rank,
                         const float4* gathered, float4* avg, uint32_t* rgb8, const PostDev* post);
struct InstSrc;
// persistent traversal grid when the stacks spill to HBM (4 waves/SIMD: 256 CUs x 4 SIMDs x 4), and the LDS
// stack levels of that form and of the one-ray query kernels (prt_traverse8.h kQueryStack)
constexpr uint32_t kSpillTraceBlocks = 256u * 4u * 4u;
constexpr int kSpillTraceStack = 18;
// device refit of the instances (prt_refit.h)
hipError_t launch_refit(hipStream_t s, const InstSrc* src, int32_t n, InstDev* out);
// the stream waits until *flag (coherent pinned host memory, device address) is nonzero; after `seconds` it stops
// waiting and sets *err (prt_render.hip k_wait_host)
hipError_t launch_wait_host(hipStream_t s, uint32_t* flag, uint32_t* err, double seconds);
hipError_t launch_primary_hits(const LaunchCfg& c, const SceneDev& S, const TileMap& M, HitOut* out, Counters* cnt);
hipError_t launch_intersect(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                            const float* tmax, HitOut* out);
hipError_t launch_occluded(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                           const float* tmax, int32_t* out);
// prt_brdf_probe: n records of 24 floats in, 8 out (include/prt.h PRT_PROBE_*)
hipError_t launch_brdf_probe(hipStream_t s, int32_t op, int32_t n, const float* in, float* out);

}  // namespace prt
