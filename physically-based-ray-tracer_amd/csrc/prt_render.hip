// prt_render.hip -- path-tracing kernels for gfx950 (MI355X).
//
// k_trace_frames: one lane = one (pixel, reference frame) work item, tracing the frame's camera
//   path(s) in the canonical order (AA jitter, Trace(r1), Trace(r2)) through
//   the restated Renderer::Trace (Core/Renderer.cpp:150-406): TLAS->BLAS closest hit, hit
//   attributes, one stochastic NEE light-class sample with shadow any-hit rays, lobe pick, BRDF
//   sampling, bounce.  The recursion `result + Trace(..) * throughput` is evaluated bottom-up from a
//   per-lane (result, throughput) stack so float rounding matches the recursive reference exactly.
// k_accumulate: per pixel, folds the frames into the persistent accumulator with the reference's
//   distance-keyed progressive mean (Core/Renderer.cpp:81-104) and packs RGB8 (precomp.h:310-315).
#include "prt_launch.h"

namespace prt {

enum : uint32_t {
  kAA = 1u << 0, kAccumulate = 1u << 1, kGamma = 1u << 2, kNormalMap = 1u << 3,
  kSkybox = 1u << 4, kLighted = 1u << 5, kStochastic = 1u << 6
};
constexpr int kMaxBounces = 16;

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

// Camera::GetPrimaryRay (Core/Camera.cpp:113-139, non-Panini branch)
__device__ __forceinline__ Ray primary_ray(const SceneDev& S, float x, float y, int W, int H) {
  const float u = x * (1.0f / (float)W);
  const float v = y * (1.0f / (float)H);
  const V3 camPos = v3(S.cam[0], S.cam[1], S.cam[2]);
  const V3 TL = v3(S.cam[3], S.cam[4], S.cam[5]), TR = v3(S.cam[6], S.cam[7], S.cam[8]),
           BL = v3(S.cam[9], S.cam[10], S.cam[11]);
  const V3 P = TL + u * (TR - TL) + v * (BL - TL);
  const V3 dir = normalize(P - camPos);
  return make_ray(camPos, dir);
}

// Renderer::Trace, iterative.  Returns radiance; *t_primary = closest-hit t of the first segment.
template <int STACK>
__device__ V3 trace_path(const SceneDev& S, const TraceArgs& A, Ray r, uint32_t& seed, float* t_primary,
                         uint32_t& nseg, uint32_t& nshadow, uint32_t* stk) {
  V3 R[kMaxBounces], T[kMaxBounces];
  int nd = 0;
  V3 Lend = v3(0.0f, 0.0f, 0.0f);
  const uint32_t fl = A.flags;
  for (int depth = 0;; depth++) {
    if (depth >= A.bounces) { Lend = v3(0.0f, 0.0f, 0.0f); break; }                   // :152
    const Hit h = scene_closest<STACK, kBlock>(S, r, kFar, stk);                         // :157
    nseg++;
    if (depth == 0 && t_primary) *t_primary = h.t;
    if (h.t >= kFar) { Lend = (fl & kSkybox) ? sample_sky(S, r.D) : v3(0.0f, 0.0f, 0.0f); break; }  // :159
    const V3 I = r.O + h.t * r.D;                                                          // tiny_bvh.h:586
    const V3 V = -r.D;
    const HitAttr ha = hit_attributes(S, h.inst, h.prim, h.u, h.v, (fl & kNormalMap) != 0);
    const V3 N = ha.N;
    const Material& m = ha.m;
    if (A.mode != 0) {                                                                     // :170-194
      switch (A.mode) {
        case 1: Lend = m.base; break;
        case 4: Lend = v3(m.metal, m.metal, m.metal); break;
        case 5: Lend = v3(m.rough, m.rough, m.rough); break;
        case 6: Lend = m.emis; break;
        case 2: {
          const V3 g = geometry_normal(S, h.inst, h.prim);
          Lend = v3(g.x + 1.0f, g.y + 1.0f, g.z + 1.0f) * 0.5f;
          break;
        }
        case 3: Lend = v3(N.x + 1.0f, N.y + 1.0f, N.z + 1.0f) * 0.5f; break;
        default: Lend = v3(0.0f, 0.0f, 0.0f); break;
      }
      break;
    }
    V3 result = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * m.emis;                  // :196
    if (fl & kStochastic) {
      const float pP = 0.3f, pD = 0.5f, pS = 0.2f;
      const float xi = random_float(seed);                                                 // :210
      const int pick = (xi < pP) ? 0 : ((xi < pP + pD) ? 1 : 2);
      if (pick == 0) {                                                                     // :216-269
        float Lx[4], Ly[4], Lz[4], dsq[4];
        V3 fc[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          Lx[i] = S.ppos[3 * i] - I.x; Ly[i] = S.ppos[3 * i + 1] - I.y; Lz[i] = S.ppos[3 * i + 2] - I.z;
          dsq[i] = (Lx[i] * Lx[i] + Ly[i] * Ly[i]) + Lz[i] * Lz[i];
          const float dist = sqrtf(dsq[i]);
          const float invD = 1.0f / dist;  // _mm_rcp_ps restated as an exact reciprocal
          Lx[i] = Lx[i] * invD; Ly[i] = Ly[i] * invD; Lz[i] = Lz[i] * invD;
          float cosa = (N.x * Lx[i] + N.y * Ly[i]) + N.z * Lz[i];
          cosa = (cosa > 0.0f) ? cosa : 0.0f;  // _mm_max_ps(cosa, 0)
          const float k = invD * cosa;
          fc[i] = v3(S.pcol[3 * i] * k, S.pcol[3 * i + 1] * k, S.pcol[3 * i + 2] * k);
        }
        V3 contrib = v3(0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const V3 L = v3(Lx[i], Ly[i], Lz[i]);
          const Ray sr = make_ray(I + L * kEpsilon, L);
          nshadow++;
          if (!scene_anyhit<STACK, kBlock>(S, sr, dsq[i] - kEpsilon, stk)) contrib = contrib + fc[i];
        }
        contrib = contrib / pP;
        const int wl = (int)(random_float(seed) * 10) % 4;                                // :267
        V3 add = v3(0.0f, 0.0f, 0.0f);
        if (fl & kLighted) {
          const float lx = wl == 0 ? Lx[0] : wl == 1 ? Lx[1] : wl == 2 ? Lx[2] : Lx[3];
          const float ly = wl == 0 ? Ly[0] : wl == 1 ? Ly[1] : wl == 2 ? Ly[2] : Ly[3];
          const float lz = wl == 0 ? Lz[0] : wl == 1 ? Lz[1] : wl == 2 ? Lz[2] : Lz[3];
          add = eval_combined_brdf(N, v3(lx, ly, lz), V, m) * contrib;
        }
        result = result + v3(1.0f, 1.0f, 1.0f) * add;
      } else {                                                                             // :270-310
        const float* lp = pick == 1 ? S.dpos : S.spos;
        const float* lc = pick == 1 ? S.dcol : S.scol;
        V3 L = v3(lp[0], lp[1], lp[2]) - I;
        const float distance = length(L);
        L = L / distance;
        const float cosa = smax(0.0f, dot(N, L));
        const Ray sr = make_ray(I + L * kEpsilon, L);
        nshadow++;
        const bool occ = scene_anyhit<STACK, kBlock>(S, sr, distance - kEpsilon, stk);
        V3 contrib = v3(0.0f, 0.0f, 0.0f);
        if (pick == 1) {
          if (!occ) contrib = v3(lc[0], lc[1], lc[2]) * cosa;
          contrib = contrib / pD;
        } else {
          const float factor = dot(L, v3(S.srot[0], S.srot[1], S.srot[2]));
          if (!occ) {
            if ((double)factor > 0.9) contrib = v3(lc[0], lc[1], lc[2]) * (1 / (distance * distance)) * cosa;
            else contrib = v3(0.0f, 0.0f, 0.0f);
          }
          contrib = contrib / pS;
        }
        V3 add = v3(0.0f, 0.0f, 0.0f);
        if (fl & kLighted) add = eval_combined_brdf(N, L, V, m) * contrib;
        result = result + v3(1.0f, 1.0f, 1.0f) * add;
      }
    } else {                                                                               // :312-326
      V3 L = v3(S.dpos[0], S.dpos[1], S.dpos[2]) - I;
      const float distance = length(L);
      L = L / distance;
      const float cosa = smax(0.0f, dot(N, L));
      const Ray sr = make_ray(I + L * kEpsilon, L);
      nshadow++;
      V3 contrib = v3(0.0f, 0.0f, 0.0f);  // uninitialised when occluded in the reference; 0 here
      if (!scene_anyhit<STACK, kBlock>(S, sr, distance - kEpsilon, stk)) contrib = v3(S.dcol[0], S.dcol[1], S.dcol[2]) * cosa;
      V3 add = v3(0.0f, 0.0f, 0.0f);
      if (fl & kLighted) add = eval_combined_brdf(N, L, V, m) * contrib;
      result = result + v3(1.0f, 1.0f, 1.0f) * add;
    }
    if (depth == A.bounces - 1) { Lend = result; break; }                                  // :329
    // :331-372 dielectric path is dead (transmissivness is never set, Scene.cpp:193-197)
    int type = 1;
    V3 thr = v3(1.0f, 1.0f, 1.0f);
    if (m.metal == 1.0f && m.rough == 0.0f) type = 2;                                      // :376
    else {
      const float bp = brdf_probability(m, V, N);                                          // :380
      if (random_float(seed) < bp) { type = 2; thr = thr / bp; }
      else { type = 1; thr = thr / (1.0f - bp); }
    }
    V3 wgt = v3(1.0f, 1.0f, 1.0f), dir;
    V2 u;
    u.x = random_float(seed);                                                              // :396
    u.y = random_float(seed);
    if (!eval_indirect_brdf(u, N, V, m, type, dir, wgt)) { Lend = result; break; }       // :398
    thr = thr * wgt;
    R[nd] = result;
    T[nd] = thr;
    nd++;
    r = make_ray(I + dir * kEpsilon, dir);                                                 // :404
  }
  V3 L = Lend;
  for (int k = nd - 1; k >= 0; k--) L = R[k] + L * T[k];
  return L;
}

template <int STACK>
__global__ void __launch_bounds__(kBlock) k_trace_frames(SceneDev S, TraceArgs A, TileMap M, float4* __restrict__ out,
                                                         Counters* __restrict__ cnt) {
  __shared__ uint32_t lds_stack[STACK * kBlock];
  uint32_t* stk = lds_stack + threadIdx.x;
  const uint64_t item = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t total = (uint64_t)M.items * (uint64_t)A.frames;
  uint32_t nseg = 0, nsh = 0;
  if (item < total) {
    const uint32_t f = (uint32_t)(item / M.items), r = (uint32_t)(item % M.items);
    int32_t x, y;
    if (item_pixel(M, r, x, y)) {
      const uint32_t p = (uint32_t)(y * A.W + x);
      uint32_t seed = init_seed(A.seed + p + (uint32_t)A.W * (uint32_t)A.H * (A.frame_index + f));
      float t1 = kFar;
      const Ray r1 = primary_ray(S, (float)x, (float)y, A.W, A.H);
      V3 res;
      if (A.flags & kAA) {                                                                 // :59-66
        const float jx = random_float(seed), jy = random_float(seed);
        const Ray r2 = primary_ray(S, (float)x + jx, (float)y + jy, A.W, A.H);
        const V3 s1 = trace_path<STACK>(S, A, r1, seed, &t1, nseg, nsh, stk);
        const V3 s2 = trace_path<STACK>(S, A, r2, seed, nullptr, nseg, nsh, stk);
        res = 0.5f * (s1 + s2);
      } else {
        res = trace_path<STACK>(S, A, r1, seed, &t1, nseg, nsh, stk);
      }
      if (A.flags & kGamma) res = v3(sqrtf(res.x), sqrtf(res.y), sqrtf(res.z));          // :73-79
      out[item] = make_float4(res.x, res.y, res.z, t1);
    } else {
      out[item] = make_float4(0.0f, 0.0f, 0.0f, kFar);
    }
  }
  wave_count(cnt, nseg, nsh);
}

// RGBF32_to_RGB8 (template/precomp.h:310-315, scalar path)
__device__ __forceinline__ uint32_t pack1(float x) {
  const float mm = smin(1.0f, x);
  return mm > 0.0f ? (uint32_t)(255.0f * mm) : 0u;
}

// Core/Renderer.cpp:81-104,137.  tiles_out != null: write the average in item (tile-compact) order.
__global__ void __launch_bounds__(kBlock) k_accumulate(TileMap M, int32_t frames, uint32_t flags,
                                                       const float4* __restrict__ fr, float4* __restrict__ acc,
                                                       int32_t* __restrict__ nsamp, float* __restrict__ dist,
                                                       float4* __restrict__ avg_out, uint32_t* __restrict__ rgb8_out,
                                                       float4* __restrict__ tiles_out) {
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
      A = make_float4(v.x, v.y, v.z, 0.0f);
      a = A;
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
                                                   uint32_t* __restrict__ rgb8_out) {
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
  if (rgb8_out) rgb8_out[p] = (pack1(a.x) << 16) + (pack1(a.y) << 8) + pack1(a.z);
}

// ---- geometry-only kernels

template <int STACK>
__global__ void __launch_bounds__(kBlock) k_primary_hits(SceneDev S, TileMap M, HitOut* __restrict__ out,
                                                         Counters* __restrict__ cnt) {
  __shared__ uint32_t lds_stack[STACK * kBlock];
  uint32_t* stk = lds_stack + threadIdx.x;
  const uint32_t r = blockIdx.x * kBlock + threadIdx.x;
  uint32_t nseg = 0;
  if (r < M.items) {
    int32_t x, y;
    if (item_pixel(M, r, x, y)) {
      const Ray ray = primary_ray(S, (float)x, (float)y, M.W, M.H);
      const Hit h = scene_closest<STACK, kBlock>(S, ray, kFar, stk);
      nseg = 1;
      HitOut o;
      o.t = h.t; o.u = h.u; o.v = h.v; o.prim = h.prim; o.inst = h.inst;
      out[(size_t)y * M.W + x] = o;
    }
  }
  wave_count(cnt, nseg, 0);
}

template <int STACK>
__global__ void __launch_bounds__(kBlock) k_intersect(SceneDev S, int32_t n, const float* __restrict__ O,
                                                      const float* __restrict__ D, const float* __restrict__ tmax,
                                                      HitOut* __restrict__ out) {
  __shared__ uint32_t lds_stack[STACK * kBlock];
  uint32_t* stk = lds_stack + threadIdx.x;
  const int32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Ray r = make_ray(v3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), v3(D[3 * i], D[3 * i + 1], D[3 * i + 2]));
  const Hit h = scene_closest<STACK, kBlock>(S, r, tmax ? tmax[i] : kFar, stk);
  HitOut o;
  o.t = h.t; o.u = h.u; o.v = h.v; o.prim = h.prim; o.inst = h.inst;
  out[i] = o;
}

template <int STACK>
__global__ void __launch_bounds__(kBlock) k_occluded(SceneDev S, int32_t n, const float* __restrict__ O,
                                                     const float* __restrict__ D, const float* __restrict__ tmax,
                                                     int32_t* __restrict__ out) {
  __shared__ uint32_t lds_stack[STACK * kBlock];
  uint32_t* stk = lds_stack + threadIdx.x;
  const int32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const Ray r = make_ray(v3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), v3(D[3 * i], D[3 * i + 1], D[3 * i + 2]));
  out[i] = scene_anyhit<STACK, kBlock>(S, r, tmax[i], stk) ? 1 : 0;
}

// ---- launchers (host)
static inline unsigned grid_of(uint64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

hipError_t launch_trace_frames(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                               float4* out, Counters* cnt) {
  const uint64_t total = (uint64_t)M.items * (uint64_t)A.frames;
  if (total == 0) return hipSuccess;
  if (c.stack <= 24)
    hipLaunchKernelGGL(k_trace_frames<24>, dim3(grid_of(total)), dim3(kBlock), 0, c.stream, S, A, M, out, cnt);
  else
    hipLaunchKernelGGL(k_trace_frames<48>, dim3(grid_of(total)), dim3(kBlock), 0, c.stream, S, A, M, out, cnt);
  return hipGetLastError();
}

hipError_t launch_accumulate(const LaunchCfg& c, const TileMap& M, int32_t frames, uint32_t flags, const float4* fr,
                             float4* acc, int32_t* nsamp, float* dist, float4* avg, uint32_t* rgb8, float4* tiles) {
  if (M.items == 0) return hipSuccess;
  hipLaunchKernelGGL(k_accumulate, dim3(grid_of(M.items)), dim3(kBlock), 0, c.stream, M, frames, flags, fr, acc, nsamp,
                     dist, avg, rgb8, tiles);
  return hipGetLastError();
}

hipError_t launch_untile(const LaunchCfg& c, int32_t W, int32_t H, int32_t ts, int32_t world, uint32_t per_rank,
                         const float4* gathered, float4* avg, uint32_t* rgb8) {
  const uint64_t n = (uint64_t)per_rank * (uint64_t)world;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_untile, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, W, H, ts, world, per_rank, gathered, avg,
                     rgb8);
  return hipGetLastError();
}

hipError_t launch_primary_hits(const LaunchCfg& c, const SceneDev& S, const TileMap& M, HitOut* out, Counters* cnt) {
  if (M.items == 0) return hipSuccess;
  if (c.stack <= 24)
    hipLaunchKernelGGL(k_primary_hits<24>, dim3(grid_of(M.items)), dim3(kBlock), 0, c.stream, S, M, out, cnt);
  else
    hipLaunchKernelGGL(k_primary_hits<48>, dim3(grid_of(M.items)), dim3(kBlock), 0, c.stream, S, M, out, cnt);
  return hipGetLastError();
}

hipError_t launch_intersect(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                            const float* tmax, HitOut* out) {
  if (n <= 0) return hipSuccess;
  if (c.stack <= 24)
    hipLaunchKernelGGL(k_intersect<24>, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, S, n, O, D, tmax, out);
  else
    hipLaunchKernelGGL(k_intersect<48>, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, S, n, O, D, tmax, out);
  return hipGetLastError();
}

hipError_t launch_occluded(const LaunchCfg& c, const SceneDev& S, int32_t n, const float* O, const float* D,
                           const float* tmax, int32_t* out) {
  if (n <= 0) return hipSuccess;
  if (c.stack <= 24)
    hipLaunchKernelGGL(k_occluded<24>, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, S, n, O, D, tmax, out);
  else
    hipLaunchKernelGGL(k_occluded<48>, dim3(grid_of(n)), dim3(kBlock), 0, c.stream, S, n, O, D, tmax, out);
  return hipGetLastError();
}

}  // namespace prt
