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
// Queues are split into kNSub sub-queues, each with its own counter on its own 128-B line, so the
// (block-aggregated, one atomic per 256 entries) appends never pile up on one address.  Consumers
// need no atomics: a block loads the kNSub counts into an LDS prefix table and walks a static,
// interleaved set of 64-entry chunks (traversal kernels use one-wave blocks, so a slow wave never
// holds back its siblings' slots).  All per-item state is SoA in HBM; no host synchronisation.
#include "prt_launch.h"
#include "prt_path.h"
#include "prt_persist.h"
#include "prt_queue.h"

namespace prt {

// ---- init: items -> primary rays, appended to queue 0 (sub-queue = block % kNSub)
__global__ void __launch_bounds__(kBlock) k_wave_init(SceneDev S, TraceArgs A, TileMap M, WaveBufs B,
                                                      float4* __restrict__ out) {
  __shared__ uint32_t sm[8];
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* cnt = qcounter(B.ctr, 0, 0, sub);
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
        enq = true;
      } else {
        out[i] = make_float4(0.0f, 0.0f, 0.0f, kFar);  // bounces == 0: Trace returns 0, t1 stays BVH_FAR
      }
    }
    const uint32_t slot = block_append(cnt, enq ? 1u : 0u, sm);
    if (enq) B.q0[sub * B.qcap + slot] = i;
  }
}

// ---- closest hit (one-wave blocks, static interleaved chunks of the live queue)
template <int BV>
__global__ void __launch_bounds__(64) k_extend(SceneDev S, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t lds_stack[Trav<BV>::kWords * 64];
  __shared__ uint32_t pref[kNSub + 1];
  uint32_t* stk = lds_stack + threadIdx.x;
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  uint32_t* fctr = fetch_counters(B.ctr, iter, 0);
  uint32_t part = xcc_id(), base = 0;
  while (fetch_chunk(fctr, total, part, base)) {
    const uint32_t g = base + threadIdx.x;
    const uint32_t hi = (uint32_t)(((uint64_t)total * (part + 1)) / kParts);
    if (g < hi) {
      const uint32_t item = q[map_slot(pref, g, B.qcap)];
      const float4 o = B.ro[item], d = B.rd[item];
      Ray r;
      r.O = v3(o.x, o.y, o.z);
      r.D = v3(d.x, d.y, d.z);
      r.rD = v3(safercp(d.x), safercp(d.y), safercp(d.z));
      const Hit h = Trav<BV>::template closest<64>(S, r, kFar, stk);
      B.hit[item] = make_float4(h.t, h.u, h.v, __uint_as_float(pack_hit(h.prim, h.inst)));
    }
  }
}

// ---- shading, NEE set-up (shadow rays straight into the shadow queue), BRDF sampling (render mode 0)
__global__ void __launch_bounds__(kBlock) k_shade(SceneDev S, TraceArgs A, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t pref[kNSub + 1];
  __shared__ uint32_t sm[8];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* shcnt = qcounter(B.ctr, iter, 1, sub);
  float4* sho = B.sho + (size_t)sub * B.scap;
  float4* shd = B.shd + (size_t)sub * B.scap;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  const uint32_t fl = A.flags;
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    uint32_t item = 0, info = 0, seed = 0, nr = 0;
    int kind = 0;
    float4 hh = make_float4(kFar, 0.0f, 0.0f, 0.0f);
    const bool active = g < total;
    if (active) {
      item = q[map_slot(pref, g, B.qcap)];
      info = B.info[item];
      hh = B.hit[item];
      if ((info & 0x1FFu) == 0) B.s1[item].w = hh.x;                                        // r1.hit.t
      if (hh.x < kFar) {  // misses (:159) are resolved in k_resolve: the sky lookup's double-precision
                          // atan2 / acos would otherwise set this kernel's register budget
        seed = B.seed[item];
        kind = nee_kind(fl, seed);                                                           // :198-214
        nr = (uint32_t)nee_rays(kind);
      }
    }
    // reserve the shadow-ray slots of the whole block at once (one atomic per 256 items)
    const uint32_t s0 = block_append(shcnt, nr, sm);
    uint32_t status = kStMiss;
    if (nr) {
      const uint32_t depth = info & 0xFFu;
      const float4 o = B.ro[item], d = B.rd[item];
      const V3 D = v3(d.x, d.y, d.z);
      const uint32_t pk = __float_as_uint(hh.w);
      const V3 I = v3(o.x, o.y, o.z) + hh.x * D;                                             // tiny_bvh.h:586
      const V3 V = -D;
      const HitAttr ha = hit_attributes(S, pk >> 26, pk & 0x03FFFFFFu, hh.y, hh.z, (fl & kNormalMap) != 0);
      const V3 e = v3(0.0f, 0.0f, 0.0f) + v3(1.0f, 1.0f, 1.0f) * ha.m.emis;                // :196
      B.ne[item] = make_float4(e.x, e.y, e.z, 0.0f);
      const V3 brdf = nee_lights(S, fl, kind, I, V, ha.N, ha.m, seed, [&](int k, const Ray& sr, float tmax, V3 fk) {
        sho[s0 + k] = make_float4(sr.O.x, sr.O.y, sr.O.z, tmax);
        shd[s0 + k] = make_float4(sr.D.x, sr.D.y, sr.D.z, __uint_as_float(4u * item + (uint32_t)k));
        B.nf[4 * (size_t)item + k] = make_float4(fk.x, fk.y, fk.z, 0.0f);
      });
      B.nb[item] = make_float4(brdf.x, brdf.y, brdf.z, 0.0f);
      B.vis[item] = 0u;
      status = kStNeeEnd;
      if ((int)depth != A.bounces - 1) {                                                     // :329
        V3 dir, thr;
        if (sample_bounce(ha.m, V, ha.N, seed, dir, thr)) {                                  // :376-399
          status = kStNeeCont;
          B.T[(size_t)depth * B.n + item] = make_float4(thr.x, thr.y, thr.z, 0.0f);
          const Ray nr2 = make_ray(I + dir * kEpsilon, dir);                                 // :404
          B.ro[item] = make_float4(nr2.O.x, nr2.O.y, nr2.O.z, 0.0f);
          B.rd[item] = make_float4(nr2.D.x, nr2.D.y, nr2.D.z, 0.0f);
        }
      }
      B.seed[item] = seed;
    }
    if (active) B.info[item] = (info & 0x1FFu) | (status << 16) | ((uint32_t)kind << 20);
  }
}

// ---- misses of this iteration (:159): sky radiance (or 0) ends the path.  Kept out of k_shade and
// k_resolve: the sky lookup's double-precision atan2 / acos would set their register budgets.
__global__ void __launch_bounds__(kBlock) k_miss(SceneDev S, TraceArgs A, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t pref[kNSub + 1];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    if (g >= total) continue;
    const uint32_t item = q[map_slot(pref, g, B.qcap)];
    const uint32_t info = B.info[item];
    if (((info >> 16) & 3u) != kStMiss) continue;
    V3 L = v3(0.0f, 0.0f, 0.0f);
    if (A.flags & kSkybox) {
      const float4 d = B.rd[item];
      L = sample_sky(S, v3(d.x, d.y, d.z));
    }
    B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
    B.info[item] = info & ~(3u << 16);  // kStEndValue
  }
}

// ---- debug render modes (Core/Renderer.cpp:170-194): the hit's debug colour ends the path
__global__ void __launch_bounds__(kBlock) k_shade_debug(SceneDev S, TraceArgs A, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t pref[kNSub + 1];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  const uint32_t fl = A.flags;
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    if (g >= total) continue;
    const uint32_t item = q[map_slot(pref, g, B.qcap)];
    const uint32_t info = B.info[item];
    const float4 hh = B.hit[item];
    if ((info & 0x1FFu) == 0) B.s1[item].w = hh.x;
    V3 L = v3(0.0f, 0.0f, 0.0f);
    if (hh.x >= kFar) {
      if (fl & kSkybox) {
        const float4 d = B.rd[item];
        L = sample_sky(S, v3(d.x, d.y, d.z));
      }
    } else {
      const uint32_t pk = __float_as_uint(hh.w);
      const HitAttr ha = hit_attributes(S, pk >> 26, pk & 0x03FFFFFFu, hh.y, hh.z, (fl & kNormalMap) != 0);
      L = debug_view(S, A.mode, ha, pk >> 26, pk & 0x03FFFFFFu);
    }
    B.ne[item] = make_float4(L.x, L.y, L.z, 0.0f);
    B.info[item] = info & 0x1FFu;  // status kStEndValue
  }
}

// ---- any hit for the shadow queue
template <int BV>
__global__ void __launch_bounds__(64) k_shadow(SceneDev S, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t lds_stack[Trav<BV>::kWords * 64];
  __shared__ uint32_t pref[kNSub + 1];
  uint32_t* stk = lds_stack + threadIdx.x;
  uint8_t* vis8 = reinterpret_cast<uint8_t*>(B.vis);
  const uint32_t total = load_prefix(B.ctr, iter, 1, pref);
  uint32_t* fctr = fetch_counters(B.ctr, iter, 1);
  uint32_t part = xcc_id(), base = 0;
  while (fetch_chunk(fctr, total, part, base)) {
    const uint32_t g = base + threadIdx.x;
    const uint32_t hi = (uint32_t)(((uint64_t)total * (part + 1)) / kParts);
    if (g < hi) {
      const uint32_t slot = map_slot(pref, g, B.scap);
      const float4 o = B.sho[slot], d = B.shd[slot];
      Ray r;
      r.O = v3(o.x, o.y, o.z);
      r.D = v3(d.x, d.y, d.z);
      r.rD = v3(safercp(d.x), safercp(d.y), safercp(d.z));
      if (!Trav<BV>::template anyhit<64>(S, r, o.w, stk)) vis8[__float_as_uint(d.w)] = 1;
    }
  }
}

// ---- persistent-lane variants (Node8): lanes refill from the queue as their rays finish (prt_persist.h)
template <bool HALF, int REFILL, int STACK, int WAVES>
__global__ void __launch_bounds__(64, WAVES) k_extend_p(SceneDev S, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t lds_stack[2 * STACK * 64];
  __shared__ uint32_t pref[kNSub + 1];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  if (blockIdx.x * 64u >= total) return;  // small queues: only as many waves as 64-ray chunks
  uint32_t* fctr = fetch_counters(B.ctr, iter, 0);
  uint32_t part = xcc_id();
  trav8_persistent<0, HALF, STACK, REFILL>(
      S, lds_stack + threadIdx.x,
      [&](uint32_t* base, uint32_t want) { return fetch_some(fctr, total, part, base, want); },
      [&](uint32_t g, V3& O, V3& D, float& tmax, bool&) -> uint32_t {
        const uint32_t item = q[map_slot(pref, g, B.qcap)];
        const float4 o = B.ro[item], d = B.rd[item];
        O = v3(o.x, o.y, o.z);
        D = v3(d.x, d.y, d.z);
        tmax = kFar;
        return item;
      },
      [&](uint32_t item, bool, V3& O, V3& D) {
        const float4 o = B.ro[item], d = B.rd[item];
        O = v3(o.x, o.y, o.z);
        D = v3(d.x, d.y, d.z);
      },
      [&](uint32_t item, const Hit& h, bool, bool) {
        B.hit[item] = make_float4(h.t, h.u, h.v, __uint_as_float(pack_hit(h.prim, h.inst)));
      });
}

template <bool HALF, int REFILL, int STACK, int WAVES>
__global__ void __launch_bounds__(64, WAVES) k_shadow_p(SceneDev S, WaveBufs B, uint32_t iter) {
  __shared__ uint32_t lds_stack[2 * STACK * 64];
  __shared__ uint32_t pref[kNSub + 1];
  uint8_t* vis8 = reinterpret_cast<uint8_t*>(B.vis);
  const uint32_t total = load_prefix(B.ctr, iter, 1, pref);
  if (blockIdx.x * 64u >= total) return;
  uint32_t* fctr = fetch_counters(B.ctr, iter, 1);
  uint32_t part = xcc_id();
  trav8_persistent<1, HALF, STACK, REFILL>(
      S, lds_stack + threadIdx.x,
      [&](uint32_t* base, uint32_t want) { return fetch_some(fctr, total, part, base, want); },
      [&](uint32_t g, V3& O, V3& D, float& tmax, bool&) -> uint32_t {
        const uint32_t slot = map_slot(pref, g, B.scap);
        const float4 o = B.sho[slot], d = B.shd[slot];
        O = v3(o.x, o.y, o.z);
        D = v3(d.x, d.y, d.z);
        tmax = o.w;
        return slot;
      },
      [&](uint32_t slot, bool, V3& O, V3& D) {
        const float4 o = B.sho[slot], d = B.shd[slot];
        O = v3(o.x, o.y, o.z);
        D = v3(d.x, d.y, d.z);
      },
      [&](uint32_t slot, const Hit&, bool, bool occluded) {
        const uint32_t tag = __float_as_uint(B.shd[slot].w);
        if (!occluded) vis8[tag] = 1;
      });
}

// ---- NEE resolve, (result, throughput) stack, path end, AA path 2, frame write
__global__ void __launch_bounds__(kBlock) k_resolve(SceneDev S, TraceArgs A, TileMap M, WaveBufs B, uint32_t iter,
                                                    float4* __restrict__ out) {
  __shared__ uint32_t pref[kNSub + 1];
  __shared__ uint32_t sm[8];
  const uint32_t* q = (iter & 1) ? B.q1 : B.q0;
  uint32_t* qn = (iter & 1) ? B.q0 : B.q1;
  const uint32_t sub = blockIdx.x % kNSub;
  uint32_t* ncnt = qcounter(B.ctr, iter + 1, 0, sub);
  const uint32_t total = load_prefix(B.ctr, iter, 0, pref);
  const uint32_t fl = A.flags;
  for (uint32_t c = blockIdx.x; c * kBlock < total; c += gridDim.x) {
    const uint32_t g = c * kBlock + threadIdx.x;
    bool enq = false;
    uint32_t item = 0;
    if (g < total) {
      item = q[map_slot(pref, g, B.qcap)];
      const uint32_t info = B.info[item];
      const uint32_t depth = info & 0xFFu, path = (info >> 8) & 1u, status = (info >> 16) & 3u,
                     kind = (info >> 20) & 3u;
      const float4 ne = B.ne[item];
      V3 L = v3(ne.x, ne.y, ne.z);
      bool path_end = true;
      if (status == kStNeeEnd || status == kStNeeCont) {
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
          const uint32_t r = (B.base + item) % M.items;
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
    const uint32_t slot = block_append(ncnt, enq ? 1u : 0u, sm);
    if (enq) qn[sub * B.qcap + slot] = item;
  }
}

// persistent traversal launch: LDS stack depth and waves/SIMD by c.occ (the BVH depth was checked against
// the stack on the host), refill threshold by c.trav; grid = the resident wave count
template <bool ANY, int REFILL, int STACK, int WAVES>
void launch_p1(const LaunchCfg& c, const SceneDev& S, const WaveBufs& B, uint32_t it) {
  const dim3 grid(256u * 4u * WAVES);
  if (c.layout == 9) {
    if (ANY) hipLaunchKernelGGL((k_shadow_p<true, REFILL, STACK, WAVES>), grid, dim3(64), 0, c.stream, S, B, it);
    else hipLaunchKernelGGL((k_extend_p<true, REFILL, STACK, WAVES>), grid, dim3(64), 0, c.stream, S, B, it);
  } else {
    if (ANY) hipLaunchKernelGGL((k_shadow_p<false, REFILL, STACK, WAVES>), grid, dim3(64), 0, c.stream, S, B, it);
    else hipLaunchKernelGGL((k_extend_p<false, REFILL, STACK, WAVES>), grid, dim3(64), 0, c.stream, S, B, it);
  }
}
template <bool ANY>
void launch_persistent(const LaunchCfg& c, const SceneDev& S, const WaveBufs& B, uint32_t it) {
  if (c.occ == 8) {
    if (c.trav == 32) launch_p1<ANY, 32, 8, 8>(c, S, B, it); else launch_p1<ANY, 16, 8, 8>(c, S, B, it);
  } else if (c.occ == 6 || c.occ == 7) {  // 7 (the merged pipeline's default): this launcher's 6-wave form
    if (c.trav == 32) launch_p1<ANY, 32, 12, 6>(c, S, B, it); else launch_p1<ANY, 16, 12, 6>(c, S, B, it);
  } else if (c.occ == 5) {
    if (c.trav == 32) launch_p1<ANY, 32, 14, 5>(c, S, B, it); else launch_p1<ANY, 16, 14, 5>(c, S, B, it);
  } else {
    if (c.trav == 32) launch_p1<ANY, 32, 18, 4>(c, S, B, it); else launch_p1<ANY, 16, 18, 4>(c, S, B, it);
  }
}

hipError_t launch_wave_init(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                            const WaveBufs& B, float4* out) {
  hipLaunchKernelGGL(k_wave_init, dim3(256u * 4u), dim3(kBlock), 0, c.stream, S, A, M, B, out);
  return hipGetLastError();
}

// ---- host launcher: the whole frame batch, no host synchronisation inside
hipError_t launch_wavefront(const LaunchCfg& c, const SceneDev& S, const TraceArgs& A, const TileMap& M,
                            const WaveBufs& B, float4* out, WaveTimers* tm) {
  if (B.n == 0) return hipSuccess;
  const unsigned gtrav = 256u * 16u;  // one-wave blocks, static interleaved chunks
  const unsigned gprod = 256u * 4u;   // producer blocks (multiple of kNSub)
  hipLaunchKernelGGL(k_wave_init, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, M, B, out);
  const uint32_t iters = (uint32_t)A.bounces * ((A.flags & kAA) ? 2u : 1u);
  for (uint32_t it = 0; it < iters; it++) {
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 0], c.stream);
    if (c.layout == 4) hipLaunchKernelGGL(k_extend<4>, dim3(gtrav), dim3(64), 0, c.stream, S, B, it);
    else if (c.trav == 1 && c.layout == 9) hipLaunchKernelGGL(k_extend<9>, dim3(gtrav), dim3(64), 0, c.stream, S, B, it);
    else if (c.trav == 1) hipLaunchKernelGGL(k_extend<8>, dim3(gtrav), dim3(64), 0, c.stream, S, B, it);
    else launch_persistent<false>(c, S, B, it);
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 1], c.stream);
    if (A.mode != 0) hipLaunchKernelGGL(k_shade_debug, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, B, it);
    else {
      hipLaunchKernelGGL(k_shade, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, B, it);
      hipLaunchKernelGGL(k_miss, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, B, it);
    }
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 2], c.stream);
    if (c.layout == 4) hipLaunchKernelGGL(k_shadow<4>, dim3(gtrav), dim3(64), 0, c.stream, S, B, it);
    else if (c.trav == 1 && c.layout == 9) hipLaunchKernelGGL(k_shadow<9>, dim3(gtrav), dim3(64), 0, c.stream, S, B, it);
    else if (c.trav == 1) hipLaunchKernelGGL(k_shadow<8>, dim3(gtrav), dim3(64), 0, c.stream, S, B, it);
    else launch_persistent<true>(c, S, B, it);
    if (tm) (void)hipEventRecord(tm->ev[4 * it + 3], c.stream);
    hipLaunchKernelGGL(k_resolve, dim3(gprod), dim3(kBlock), 0, c.stream, S, A, M, B, it, out);
  }
  if (tm) tm->iters = iters;
  return hipGetLastError();
}

}  // namespace prt
