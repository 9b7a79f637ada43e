// prt_render.hip -- accumulation / untile / screen-pass / geometry-query kernels (gfx950).
//
// k_accumulate: per pixel, folds the frames into the persistent accumulator with the reference's
//   distance-keyed progressive mean (Core/Renderer.cpp:81-104) and packs RGB8 (precomp.h:310-315).
#include "prt_launch.h"
#include "prt_refit.h"
#include "prt_path.h"

namespace prt {

__device__ __forceinline__ void wave_count(Counters* c, uint32_t seg, uint32_t sh) {
  // one atomic per wave: reduce across the 64 lanes first
  for (int off = 32; off > 0; off >>= 1) {
    seg += __shfl_xor(seg, off, 64);
    sh += __shfl_xor(sh, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&c->segments, (unsigned long long)seg);
    atomicAdd(&c->shadow, (unsigned long long)sh);
  }
}

// Core/Renderer.cpp:81-104,137.  tiles_out != null: write the average in item (tile-compact) order.
// totals != null: the first wave also adds this pass's ray counts (the closest / shadow queue counters of its
// `iters` wavefront iterations) to the context's running totals (prt_ray_totals), so a caller can count rays
// without a host sync per frame
__global__ void __launch_bounds__(kBlock) k_accumulate(TileMap M, int32_t frames, uint32_t flags,
                                                       const float4* __restrict__ fr, float4* __restrict__ acc,
                                                       int32_t* __restrict__ nsamp, float* __restrict__ dist,
                                                       float4* __restrict__ avg_out, uint32_t* __restrict__ rgb8_out,
                                                       float4* __restrict__ tiles_out, float4* __restrict__ acc_prev,
                                                       const uint32_t* __restrict__ ctr, uint32_t iters,
                                                       Counters* __restrict__ totals) {
  if (totals && blockIdx.x == 0 && threadIdx.x < 64) {
    unsigned long long seg = 0, sh = 0;
    for (uint32_t j = threadIdx.x; j < (iters + 2u) * kNSub; j += 64) {  // (+2: P(iters + 1) holds the merged path-2 primaries)
      const uint32_t k = j / kNSub, s = j % kNSub;
      seg += ctr[((k * 2u + 0u) * kNSub + s) * kCtrStride];
      sh += ctr[((k * 2u + 1u) * kNSub + s) * kCtrStride];
    }
    for (int off = 32; off > 0; off >>= 1) {
      seg += __shfl_xor(seg, off, 64);
      sh += __shfl_xor(sh, off, 64);
    }
    if (threadIdx.x == 0) {
      atomicAdd(&totals->segments, seg);
      atomicAdd(&totals->shadow, sh);
    }
  }
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  if (r >= M.items) return;
  int32_t x, y;
  const bool valid = item_pixel(M, r, x, y);
  if (!valid) {
    if (tiles_out) tiles_out[r] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    return;
  }
  const uint32_t p = (uint32_t)(y * M.W + x);
  float4 A = acc[p];
  int32_t n = nsamp[p];
  float d = dist[p];
  float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  for (int32_t f = 0; f < frames; f++) {
    const float4 v = fr[(size_t)f * M.items + r];
    const float t1 = v.w;
    if (acc_prev && f == frames - 1) acc_prev[p] = A;  // what the screen pass sees right of the pixel
    if (flags & kAccumulate) {
      if (fabsf(d - t1) < kEpsilon) {
        n++;
        A.x += v.x; A.y += v.y; A.z += v.z;
        const float inv = 1.f / (float)n;
        a = make_float4(A.x * inv, A.y * inv, A.z * inv, A.w * inv);
      } else {
        n = 1;
        A = make_float4(v.x, v.y, v.z, 0.0f);
        a = A;
      }
      d = t1;
    } else {
      a = make_float4(v.x, v.y, v.z, 0.0f);
      A = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // !accumulates: memset after the frame (:147)
    }
  }
  acc[p] = A;
  nsamp[p] = n;
  dist[p] = d;
  if (avg_out) avg_out[p] = a;
  if (rgb8_out) rgb8_out[p] = (pack1(a.x) << 16) + (pack1(a.y) << 8) + pack1(a.z);
  if (tiles_out) tiles_out[r] = a;
}

// rank-0 untile of the gathered tile buffers (one item = one gathered element)
__global__ void __launch_bounds__(kBlock) k_untile(int32_t W, int32_t H, int32_t ts, int32_t world, uint32_t per_rank,
                                                   const float4* __restrict__ gathered, float4* __restrict__ avg_out,
                                                   uint32_t* __restrict__ rgb8_out, PostDev post, int32_t use_post) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (uint64_t)per_rank * (uint64_t)world) return;
  const int32_t rank = (int32_t)(i / per_rank);
  const uint32_t r = (uint32_t)(i % per_rank);
  const TileMap M = make_tilemap(W, H, ts, rank, world);
  if (r >= M.items) return;
  int32_t x, y;
  if (!item_pixel(M, r, x, y)) return;
  const float4 a = gathered[i];
  const uint32_t p = (uint32_t)(y * W + x);
  if (avg_out) avg_out[p] = a;
  if (rgb8_out) {
    float4 c = a;
    if (use_post) {  // Core/Renderer.cpp:121-133 without aberration
      const float vig = vignette(post, x, y);
      c = make_float4(c.x * post.grade[0] * vig, c.y * post.grade[1] * vig, c.z * post.grade[2] * vig, 0.0f);
    }
    rgb8_out[p] = (pack1(c.x) << 16) + (pack1(c.y) << 8) + pack1(c.z);
  }
}

// Renderer::Tick's screen pass (Core/Renderer.cpp:107-133) over the whole image: chromatic aberration from
// the accumulator -- the reference walks each row left to right, so a neighbour left of x already holds
// this frame's accumulator (acc_new) and one right of x the state before it (acc_old) -- divided by this
// pixel's sample count, then colour grading and the vignette, RGBF32_to_RGB8
__global__ void __launch_bounds__(kBlock) k_postfx(PostDev P, const float4* __restrict__ acc_new,
                                                   const float4* __restrict__ acc_old, const int32_t* __restrict__ nsamp,
                                                   const float4* __restrict__ avg, uint32_t* __restrict__ rgb8_out) {
  const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
  if (p >= (uint32_t)P.W * (uint32_t)P.H) return;
  const int32_t x = (int32_t)(p % (uint32_t)P.W), y = (int32_t)(p / (uint32_t)P.W);
  const float4 a = avg[p];
  float4 c = a;
  if (P.aberration != 0) {
    const int32_t xr = max(0, min(x + P.aberration, P.W - 1)), xb = max(0, min(x - P.aberration, P.W - 1));
    const float inv = 1.f / (float)nsamp[p];
    const uint32_t row = (uint32_t)y * (uint32_t)P.W;
    const float4 R = xr <= x ? acc_new[row + xr] : acc_old[row + xr];
    const float4 B = xb <= x ? acc_new[row + xb] : acc_old[row + xb];
    const float red = 0.75f * a.x + 0.25f * (R.x * inv);
    const float blue = 0.75f * a.z + 0.25f * (B.z * inv);
    c = make_float4(red, a.y, blue, a.w);
  }
  const float vig = vignette(P, x, y);
  c = make_float4(c.x * P.grade[0], c.y * P.grade[1], c.z * P.grade[2], c.w * P.grade[3]);
  c = make_float4(c.x * vig, c.y * vig, c.z * vig, c.w * vig);
  rgb8_out[p] = (pack1(c.x) << 16) + (pack1(c.y) << 8) + pack1(c.z);
}

// ---- geometry-only kernels

__global__ void __launch_bounds__(kBlock) k_primary_hits(SceneDev S, TileMap M, HitOut* __restrict__ out,
                                                         Counters* __restrict__ cnt) {
  __shared__ uint32_t lds_stack[kQueryWords * kBlock];
  const LaneStack stk = lane_stack<kQueryStack, kBlock>(S, lds_stack + threadIdx.x);
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  uint32_t nseg = 0;
  if (r < M.items) {
    int32_t x, y;
    if (item_pixel(M, r, x, y)) {
      const Ray ray = primary_ray(S, (float)x, (float)y, M.W, M.H);
      const Hit h = scene_closest8<kQueryStack, kBlock>(S, ray, kFar, stk);
      nseg = 1;
      HitOut o;
      o.t = h.t; o.u = h.u; o.v = h.v; o.prim = h.prim; o.inst = h.inst;
      out[(size_t)y * M.W + x] = o;
    }
  }
  wave_count(cnt, nseg, 0);
}

__global__ void __launch_bounds__(kBlock) k_intersect(SceneDev S, int32_t n, const float* __restrict__ O,
                                                      const float* __restrict__ D, const float* __restrict__ tmax,
                                                      HitOut* __restrict__ out) {
  __shared__ uint32_t lds_stack[kQueryWords * kBlock];
  const LaneStack stk = lane_stack<kQueryStack, kBlock>(S, lds_stack + threadIdx.x);
  const int32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Ray r = make_ray(v3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), v3(D[3 * i], D[3 * i + 1], D[3 * i + 2]));
  const Hit h = scene_closest8<kQueryStack, kBlock>(S, r, tmax ? tmax[i] : kFar, stk);
  HitOut o;
  o.t = h.t; o.u = h.u; o.v = h.v; o.prim = h.prim; o.inst = h.inst;
  out[i] = o;
}

__global__ void __launch_bounds__(kBlock) k_occluded(SceneDev S, int32_t n, const float* __restrict__ O,
                                                     const float* __restrict__ D, const float* __restrict__ tmax,
                                                     int32_t* __restrict__ out) {
  __shared__ uint32_t lds_stack[kQueryWords * kBlock];
  const LaneStack stk = lane_stack<kQueryStack, kBlock>(S, lds_stack + threadIdx.x);
  const int32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Ray r = make_ray(v3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), v3(D[3 * i], D[3 * i + 1], D[3 * i + 2]));
  out[i] = scene_anyhit8<kQueryStack, kBlock>(S, r, tmax[i], stk) ? 1 : 0;
}

// zero two word ranges in one launch (a call's queue counters and fetch counters: one dispatch instead of two fills)
__global__ void __launch_bounds__(kBlock) k_clear2(uint32_t* __restrict__ a, uint32_t na, uint32_t* __restrict__ b,
                                                  uint32_t nb) {
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < na + nb; i += gridDim.x * kBlock) {
    if (i < na) a[i] = 0u;
    else b[i - na] = 0u;
  }
}

// ---- launchers (host)
static inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

hipError_t launch_clear2(const LaunchCfg& c, uint32_t* a, uint32_t na, uint32_t* b, uint32_t nb) {
  const uint64_t n = (uint64_t)na + nb;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_clear2, dim3((unsigned)std::min<uint64_t>(grid_of(n), 256)), dim3(kBlock), 0, c.stream, a, na, b, nb);
  return hipGetLastError();
}


hipError_t launch_accumulate(const LaunchCfg& c, const TileMap& M, int32_t frames, uint32_t flags, const float4* fr,
                             float4* acc, int32_t* nsamp, float* dist, float4* avg, uint32_t* rgb8, float4* tiles,
                             float4* acc_prev, const uint32_t* ctr, uint32_t iters, Counters* totals) {
  if (M.items == 0) return hipSuccess;
  hipLaunchKernelGGL(k_accumulate, dim3(grid_of(M.items)), dim3(kBlock), 0, c.stream, M, frames, flags, fr, acc, nsamp,
                     dist, avg, rgb8, tiles, acc_prev, ctr, iters, totals);
  return hipGetLastError();
}

hipError_t launch_postfx(const LaunchCfg& c, const PostDev& P, const float4* acc_new, const float4* acc_old,
                         const int32_t* nsamp, const float4* avg, uint32_t* rgb8) {
  const uint64_t n = (uint64_t)P.W * (uint64_t)P.H;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_postfx, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, P, acc_new, acc_old, nsamp, avg, rgb8);
  return hipGetLastError();
}

hipError_t launch_untile(const LaunchCfg& c, int32_t W, int32_t H, int32_t ts, int32_t world, uint32_t per_rank,
                         const float4* gathered, float4* avg, uint32_t* rgb8, const PostDev* post) {
  const uint64_t n = (uint64_t)per_rank * (uint64_t)world;
  if (n == 0) return hipSuccess;
  const PostDev none{};
  hipLaunchKernelGGL(k_untile, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, W, H, ts, world, per_rank, gathered, avg,
                     rgb8, post ? *post : none, post ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_primary_hits(const LaunchCfg& c, const SceneDev& S, const TileMap& M, HitOut* out, Counters* cnt) {
  if (M.items == 0) return hipSuccess;
  hipLaunchKernelGGL(k_primary_hits, dim3(grid_of(M.items)), dim3(kBlock), 0, c.stream, S, M, out, cnt);
  return hipGetLastError();
}

hipError_t launch_intersect(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                            const float* tmax, HitOut* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_intersect, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, S, n, O, D, tmax, out);
  return hipGetLastError();
}

hipError_t launch_occluded(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                           const float* tmax, int32_t* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_occluded, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, S, n, O, D, tmax, out);
  return hipGetLastError();
}

// ---- BRDF probe (prt_brdf_probe): the shading kernels' own device functions (prt_shade.h) on one record per thread
__global__ void __launch_bounds__(kBlock) k_brdf_probe(int32_t op, int32_t n, const float* __restrict__ in,
                                                       float* __restrict__ out) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const float* a = in + 24 * (size_t)i;
  float* o = out + 8 * (size_t)i;
  for (int k = 0; k < 8; k++) o[k] = 0.0f;
  const V3 N = v3(a[0], a[1], a[2]), L = v3(a[3], a[4], a[5]), V = v3(a[6], a[7], a[8]);
  Material m;
  m.base = v3(a[9], a[10], a[11]);
  m.metal = a[12];
  m.emis = v3(a[13], a[14], a[15]);
  m.rough = a[16];
  switch (op) {
    case 0: {  // PRT_PROBE_EVAL
      const V3 r = eval_combined_brdf(N, L, V, m);
      o[0] = r.x; o[1] = r.y; o[2] = r.z;
      break;
    }
    case 1:  // PRT_PROBE_PROBABILITY
      o[0] = brdf_probability(m, V, N);
      break;
    case 2: {  // PRT_PROBE_INDIRECT
      V3 dir = v3(0.0f, 0.0f, 0.0f), w = v3(1.0f, 1.0f, 1.0f);
      V2 u;
      u.x = a[17]; u.y = a[18];
      const bool ok = eval_indirect_brdf(u, N, V, m, (int)a[19], dir, w);
      o[0] = ok ? 1.0f : 0.0f;
      o[1] = dir.x; o[2] = dir.y; o[3] = dir.z;
      o[4] = w.x; o[5] = w.y; o[6] = w.z;
      break;
    }
    case 3:  // PRT_PROBE_GGX_D
      o[0] = ggx_d(a[0], a[1]);
      break;
    case 4:  // PRT_PROBE_SMITH_G2
      o[0] = smith_g2_lagarde(a[0], a[1], a[2]);
      break;
    case 5: {  // PRT_PROBE_FRESNEL
      const V3 F = fresnel_schlick(v3(a[0], a[1], a[2]), a[3], a[4]);
      o[0] = F.x; o[1] = F.y; o[2] = F.z;
      break;
    }
    case 6:  // PRT_PROBE_SHADOWED_F90
      o[0] = shadowed_f90(v3(a[0], a[1], a[2]));
      break;
    case 7: {  // PRT_PROBE_VNDF
      V2 u;
      u.x = a[5]; u.y = a[6];
      const V3 H = sample_ggx_vndf(v3(a[0], a[1], a[2]), a[3], a[4], u);
      o[0] = H.x; o[1] = H.y; o[2] = H.z;
      break;
    }
    default:
      break;
  }
}
hipError_t launch_brdf_probe(hipStream_t s, int32_t op, int32_t n, const float* in, float* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_brdf_probe, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, op, n, in, out);
  return hipGetLastError();
}

// ---- the stream's wait for a host producer (prt_api.cpp ensure_instances: the worker thread's build of the instance
// BVH, written into pinned memory before its upload): one lane polls a word of coherent pinned host memory until the
// producer sets it, sleeping between polls.  A kernel, not a host function: work enqueued behind a pending host
// function blocks the enqueuing thread on this runtime, a kernel does not.  After `limit` wall-clock ticks it gives
// up and flags err (device memory), so a producer that never comes cannot hold the GPU.
__global__ void k_wait_host(uint32_t* flag, uint32_t* err, uint64_t limit) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
    if (wall_clock64() - t0 > limit) {
      *err = 1u;
      return;
    }
    __builtin_amdgcn_s_sleep(32);
  }
}
hipError_t launch_wait_host(hipStream_t s, uint32_t* flag, uint32_t* err, double seconds) {
  int dev = 0, khz = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess) return e;
  const uint64_t limit = (uint64_t)(seconds * 1e3 * (double)(khz > 0 ? khz : 100000));
  hipLaunchKernelGGL(k_wait_host, dim3(1), dim3(64), 0, s, flag, err, limit);
  return hipGetLastError();
}

// ---- instance refit (BLASInstance::Update on the device): one thread per instance
__global__ void k_refit(const InstSrc* __restrict__ src, int32_t n, InstDev* __restrict__ out) {
  const int32_t i = (int32_t)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  InstDev I;
  refit_instance(src[i], I);
  out[i] = I;
}

hipError_t launch_refit(hipStream_t s, const InstSrc* src, int32_t n, InstDev* out) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_refit, dim3((n + 63) / 64), dim3(64), 0, s, src, n, out);
  return hipGetLastError();
}

}  // namespace prt
