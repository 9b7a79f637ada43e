// prt_wave.hip -- wavefront path tracer (default pipeline) for gfx950.
//
// The reference's recursive per-pixel Renderer::Trace (Core/Renderer.cpp:150-406) is re-cut into
// stages over a queue of live work items (one item = one pixel x reference frame, tracing its AA
// path pair sequentially so the canonical RNG stream of SURVEY Appendix B is preserved):
//
//   k_wave_init  seeds, AA jitter, primary ray r1 -> queue 0                  (:58-61)
//   per iteration (at most bounces x paths-per-frame iterations):
//     k_extend   closest hit for every queued ray (lean traversal kernel)     (:157)
//     k_shade    hit attributes, debug views, NEE set-up + shadow-ray queue,  (:159-326, 376-404)
//                lobe pick and BRDF sampling of the continuation ray
//     k_shadow   any-hit for every queued shadow ray -> visibility bytes      (:259, 278, 299, 321)
//     k_resolve  result_d from visibility, (result, throughput) stack, path end: bottom-up
//                `result + L * throughput`, AA path 2 start, gamma, frame write (:65-79, 404)
//
// Traversal kernels are persistent: each wave pulls 64 rays at a time from a device counter, so no
// host round trip is needed to size grids and slow rays do not hold a whole launch.  Queue appends
// are wave-aggregated (ballot + one atomic per wave).  All per-item state is SoA in HBM.
#include "prt_launch.h"
#include "prt_path.h"

namespace prt {

enum : uint32_t { kStEndValue = 0, kStNeeEnd = 1, kStNeeCont = 2 };

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// wave-aggregated append of `n` (0..4) entries per lane; returns this lane's first slot
__device__ __forceinline__ uint32_t wave_append(uint32_t* counter, uint32_t n) {
  const uint64_t b1 = __ballot(n & 1u), b2 = __ballot((n >> 1) & 1u), b4 = __ballot((n >> 2) & 1u);
  const uint64_t lt = (1ull << lane_id()) - 1ull;
  const uint32_t before = (uint32_t)__popcll(b1 & lt) + 2u * (uint32_t)__popcll(b2 & lt) + 4u * (uint32_t)__popcll(b4 & lt);
  const uint32_t total = (uint32_t)__popcll(b1) + 2u * (uint32_t)__popcll(b2) + 4u * (uint32_t)__popcll(b4);
  uint32_t base = 0;
  if (lane_id() == 0 && total) base = atomicAdd(counter, total);
  base = __shfl(base, 0, 64);
  return base + before;
}

__device__ __forceinline__ uint32_t pack_hit(uint32_t prim, uint32_t inst) { return prim | (inst << 26); }

__global__ void __launch_bounds__(kBlock) k_wave_init(SceneDev S, TraceArgs A, TileMap M, WaveBufs B,
                                                      float4* __restrict__ out) {
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t i0 = blockIdx.x * kBlock + (threadIdx.x & ~63u); i0 < B.n; i0 += stride) {
    const uint32_t i = i0 + lane_id();
    bool enq = false;
    if (i < B.n) {
      const uint32_t f = i / M.items, r = i % M.items;
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
        enq = true;
      } else {
        out[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);  // bounces == 0: Trace returns 0, t1 stays BVH_FAR
      }
    }
    const uint32_t slot = wave_append(&B.ctr[0], enq ? 1u : 0u);
    if (enq) B.q0[slot] = i;
  }
}

template <int STACK>
__global__ void __launch_bounds__(kBlock) k_extend(SceneDev S, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t lds_stack[STACK * kBlock];
  uint32_t* stk = lds_stack + threadIdx.x;
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t count = B.ctr[4 * iter + 0];
  while (true) {
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&B.ctr[4 * iter + 2], 64u);
    base = __shfl(base, 0, 64);
    if (base >= count) break;
    const uint32_t idx = base + lane_id();
    if (idx < count) {
      const uint32_t item = q[idx];
      const float4 o = B.ro[item], d = B.rd[item];
      Ray r;
      r.O = v3(o.x, o.y, o.z);
      r.D = v3(d.x, d.y, d.z);
      r.rD = v3(safercp(d.x), safercp(d.y), safercp(d.z));
      const Hit h = scene_closest<STACK, kBlock>(S, r, kFar, stk);
      B.hit[item] = make_float4(h.t, h.u, h.v, __uint_as_float(pack_hit(h.prim, h.inst)));
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_shade(SceneDev S, TraceArgs A, WaveBufs B, uint32_t iter) {
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t count = B.ctr[4 * iter + 0];
  const uint32_t fl = A.flags;
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t i0 = blockIdx.x * kBlock + (threadIdx.x & ~63u); i0 < count; i0 += stride) {
    const uint32_t idx = i0 + lane_id();
    uint32_t nrays = 0, item = 0;
    NeeSetup ns;
    if (idx < count) {
      item = q[idx];
      uint32_t info = B.info[item];
      const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u;
      const float4 o = B.ro[item], d = B.rd[item], hh = B.hit[item];
      const V3 O = v3(o.x, o.y, o.z), D = v3(d.x, d.y, d.z);
      if (depth == 0 && path == 0) B.s1[item].w = hh.x;                                    // r1.hit.t
      uint32_t status = kStEndValue, kind = 0;
      if (hh.x >= kFar) {                                                                    // :159
        const V3 L = (fl & kSkybox) ? sample_sky(S, D) : v3(0.0f, 0.0f, 0.0f);
        B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
      } else {
        const uint32_t pk = __float_as_uint(hh.w);
        const uint32_t prim = pk & 0x03FFFFFFu, inst = pk >> 26;
        const V3 I = O + hh.x * D;                                                           // tiny_bvh.h:586
        const V3 V = -D;
        const HitAttr ha = hit_attributes(S, inst, prim, hh.y, hh.z, (fl & kNormalMap) != 0);
        if (A.mode != 0) {
          const V3 L = debug_view(S, A.mode, ha, inst, prim);
          B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
        } else {
          uint32_t seed = B.seed[item];
          const V3 e = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * ha.m.emis;            // :196
          ns = nee_setup(S, fl, I, V, ha.N, ha.m, seed);
          nrays = (uint32_t)ns.nrays;
          kind = (uint32_t)ns.kind;
          B.ne[item] = make_float4(e.x, e.y, e.z, 0.0f);
          B.nb[item] = make_float4(ns.brdf.x, ns.brdf.y, ns.brdf.z, 0.0f);
          for (uint32_t k = 0; k < nrays; k++) B.nf[4 * (size_t)item + k] = make_float4(ns.f[k].x, ns.f[k].y, ns.f[k].z, 0.0f);
          B.vis[item] = 0u;
          status = kStNeeEnd;
          if ((int)depth != A.bounces - 1) {                                                 // :329
            V3 dir, thr;
            if (sample_bounce(ha.m, V, ha.N, seed, dir, thr)) {
              status = kStNeeCont;
              B.T[(size_t)depth * B.n + item] = make_float4(thr.x, thr.y, thr.z, 0.0f);
              const Ray nr = make_ray(I + dir * kEpsilon, dir);                              // :404
              B.ro[item] = make_float4(nr.O.x, nr.O.y, nr.O.z, 0.0f);
              B.rd[item] = make_float4(nr.D.x, nr.D.y, nr.D.z, 0.0f);
            }
          }
          B.seed[item] = seed;
        }
      }
      info = (info & 0x1FFu) | (status << 16) | (kind << 20);
      B.info[item] = info;
    }
    const uint32_t s = wave_append(&B.ctr[4 * iter + 1], nrays);
    for (uint32_t k = 0; k < nrays; k++) {
      B.sho[s + k] = make_float4(ns.ray[k].O.x, ns.ray[k].O.y, ns.ray[k].O.z, ns.tmax[k]);
      B.shd[s + k] = make_float4(ns.ray[k].D.x, ns.ray[k].D.y, ns.ray[k].D.z, __uint_as_float(4u * item + k));
    }
  }
}

template <int STACK>
__global__ void __launch_bounds__(kBlock) k_shadow(SceneDev S, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t lds_stack[STACK * kBlock];
  uint32_t* stk = lds_stack + threadIdx.x;
  const uint32_t count = B.ctr[4 * iter + 1];
  uint8_t* vis8 = reinterpret_cast<uint8_t*>(B.vis);
  while (true) {
    uint32_t base = 0;
    if (lane_id() == 0) base = atomicAdd(&B.ctr[4 * iter + 3], 64u);
    base = __shfl(base, 0, 64);
    if (base >= count) break;
    const uint32_t idx = base + lane_id();
    if (idx < count) {
      const float4 o = B.sho[idx], d = B.shd[idx];
      Ray r;
      r.O = v3(o.x, o.y, o.z);
      r.D = v3(d.x, d.y, d.z);
      r.rD = v3(safercp(d.x), safercp(d.y), safercp(d.z));
      if (!scene_anyhit<STACK, kBlock>(S, r, o.w, stk)) vis8[__float_as_uint(d.w)] = 1;
    }
  }
}

__global__ void __launch_bounds__(kBlock) k_resolve(SceneDev S, TraceArgs A, TileMap M, WaveBufs B, uint32_t iter,
                                                    float4* __restrict__ out) {
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  uint32_t* qn = (iter & 1) ? B.q0 : B.q1;
  const uint32_t count = B.ctr[4 * iter + 0];
  const uint32_t fl = A.flags;
  const uint32_t stride = gridDim.x * kBlock;
  for (uint32_t i0 = blockIdx.x * kBlock + (threadIdx.x & ~63u); i0 < count; i0 += stride) {
    const uint32_t idx = i0 + lane_id();
    bool enq = false;
    uint32_t item = 0;
    if (idx < count) {
      item = q[idx];
      const uint32_t info = B.info[item];
      const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u, status = (info >> 16) & 3u,
                     kind = (info >> 20) & 3u;
      const float4 ne = B.ne[item];
      V3 L = v3(ne.x, ne.y, ne.z);
      bool path_end = true;
      if (status != kStEndValue) {
        const float4 nb = B.nb[item];
        const uint32_t vw = B.vis[item];
        const uint32_t vis = ((vw & 0xFFu) ? 1u : 0u) | ((vw & 0xFF00u) ? 2u : 0u) | ((vw & 0xFF0000u) ? 4u : 0u) |
                             ((vw & 0xFF000000u) ? 8u : 0u);
        V3 f[4];
        const uint32_t nr = kind == 0 ? 4u : 1u;
        for (uint32_t k = 0; k < 4; k++) {
          if (k < nr) {
            const float4 fk = B.nf[4 * (size_t)item + k];
            f[k] = v3(fk.x, fk.y, fk.z);
          } else {
            f[k] = v3(0.0f, 0.0f, 0.0f);
          }
        }
        const V3 result = nee_resolve((int)kind, vis, L, v3(nb.x, nb.y, nb.z), f, fl);
        if (status == kStNeeCont) {
          B.R[(size_t)depth * B.n + item] = make_float4(result.x, result.y, result.z, 0.0f);
          B.info[item] = (depth + 1u) | (path << 8);
          enq = true;
          path_end = false;
        } else {
          L = result;
        }
      }
      if (path_end) {
        for (int k = (int)depth - 1; k >= 0; k--) {                                          // result + Trace(..) * throughput
          const float4 Rk = B.R[(size_t)k * B.n + item], Tk = B.T[(size_t)k * B.n + item];
          L = v3(Rk.x, Rk.y, Rk.z) + L * v3(Tk.x, Tk.y, Tk.z);
        }
        const float4 s1 = B.s1[item];
        if (path == 0 && (fl & kAA)) {                                                       // start Trace(r2)
          B.s1[item] = make_float4(L.x, L.y, L.z, s1.w);
          const uint32_t r = item % M.items;
          int32_t x, y;
          item_pixel(M, r, x, y);
          const float2 j = B.jit[item];
          const Ray r2 = primary_ray(S, (float)x + j.x, (float)y + j.y, A.W, A.H);
          B.ro[item] = make_float4(r2.O.x, r2.O.y, r2.O.z, 0.0f);
          B.rd[item] = make_float4(r2.D.x, r2.D.y, r2.D.z, 0.0f);
          B.info[item] = 1u << 8;
          enq = true;
        } else {
          V3 res = (fl & kAA) ? 0.5f * (v3(s1.x, s1.y, s1.z) + L) : L;                       // :65
          if (fl & kGamma) res = v3(sqrtf(res.x), sqrtf(res.y), sqrtf(res.z));              // :73-79
          out[item] = make_float4(res.x, res.y, res.z, s1.w);
        }
      }
    }
    const uint32_t slot = wave_append(&B.ctr[4 * (iter + 1) + 0], enq ? 1u : 0u);
    if (enq) qn[slot] = item;
  }
}

// ---- host launcher: the whole frame batch, no host synchronisation inside
static inline unsigned blocks_for(uint64_t n, unsigned cap) {
  const uint64_t b = (n + kBlock - 1) / kBlock;
  return (unsigned)(b < cap ? (b ? b : 1) : cap);
}

hipError_t launch_wavefront(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                            const WaveBufs& B, float4* out, WaveTimers* tm) {
  if (B.n == 0) return hipSuccess;
  const unsigned persist = 256u * 8u;  // persistent traversal grid (waves pull work from a counter)
  const unsigned gs = blocks_for(B.n, 4096u);
  hipLaunchKernelGGL(k_wave_init, dim3(gs), dim3(kBlock), 0, c.stream, S, A, M, B, out);
  const uint32_t iters = (uint32_t)A.bounces * ((A.flags & kAA) ? 2u : 1u);
  for (uint32_t it = 0; it < iters; it++) {
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 0], c.stream);
    if (c.stack <= 24) hipLaunchKernelGGL(k_extend<24>, dim3(persist), dim3(kBlock), 0, c.stream, S, B, it);
    else hipLaunchKernelGGL(k_extend<48>, dim3(persist), dim3(kBlock), 0, c.stream, S, B, it);
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 1], c.stream);
    hipLaunchKernelGGL(k_shade, dim3(gs), dim3(kBlock), 0, c.stream, S, A, B, it);
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 2], c.stream);
    if (c.stack <= 24) hipLaunchKernelGGL(k_shadow<24>, dim3(persist), dim3(kBlock), 0, c.stream, S, B, it);
    else hipLaunchKernelGGL(k_shadow<48>, dim3(persist), dim3(kBlock), 0, c.stream, S, B, it);
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 3], c.stream);
    hipLaunchKernelGGL(k_resolve, dim3(gs), dim3(kBlock), 0, c.stream, S, A, M, B, it, out);
  }
  if (tm) tm->iters = iters;
  return hipGetLastError();
}

}  // namespace prt
