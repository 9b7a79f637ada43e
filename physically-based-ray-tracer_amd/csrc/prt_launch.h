// prt_launch.h -- host-side launchers implemented in prt_render.hip.
#pragma once
#include <hip/hip_runtime.h>

#include "prt_kernels.h"

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
  int stack;  // LDS stack entries per lane: 24 or 48
};

hipError_t launch_trace_frames(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                               float4* out, Counters* cnt);
hipError_t launch_accumulate(const LaunchCfg& c, const TileMap& M, int32_t frames, uint32_t flags, const float4* fr,
                             float4* acc, int32_t* nsamp, float* dist, float4* avg, uint32_t* rgb8, float4* tiles);
hipError_t launch_untile(const LaunchCfg& c, int32_t W, int32_t H, int32_t ts, int32_t world, uint32_t per_rank,
                         const float4* gathered, float4* avg, uint32_t* rgb8);
hipError_t launch_primary_hits(const LaunchCfg& c, const SceneDev& S, const TileMap& M, HitOut* out, Counters* cnt);
hipError_t launch_intersect(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                            const float* tmax, HitOut* out);
hipError_t launch_occluded(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                           const float* tmax, int32_t* out);

}  // namespace prt
