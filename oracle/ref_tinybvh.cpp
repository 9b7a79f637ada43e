// oracle/ref_tinybvh.cpp -- TEST INFRASTRUCTURE ONLY (built into oracle/_ref/, never shipped).
//
// Compiles the reference's own vendored tinybvh v1.4.2 (/root/reference/Core/tiny_bvh.h,
// unmodified, included in place from the reference tree) and drives it exactly as the
// reference does:
//   * one BVH8_CPU per model, BuildHQ over the fat-triangle array   (Core/Model.cpp:15-16)
//   * a TLAS: BVH::Build(BLASInstance*, n, BVHBase**, n)            (Core/Scene.cpp:220-223)
//   * closest hit: tlas.Intersect(ray) -> IntersectTLAS             (Core/Renderer.cpp:157)
//   * any hit:     tlas.IsOccluded(ray) -> IsOccludedTLAS           (Core/Scene.cpp:41-45)
// The reference builds with Tmpl8 vector types (Core/tinyBVH.h:1-13); the layouts are
// identical, so tinybvh's default types are used here.  tiny_bvh.h:586 (an author-added
// member) names 'float3', hence the alias below.
//
// It also exposes a scalar re-walk of BVH8_CPU::Intersect's traversal order that counts
// interior-node and leaf visits (N_int, N_leaf for the roofline bytes);
// tests check its step count equals the library's own return value ray by ray.
#include <cstdint>
#include <cstring>
#include <vector>
namespace tinybvh { struct bvhvec3; }
using float3 = tinybvh::bvhvec3;
#define private public    // harness-only: read BVH8_CPU's node arrays for the visit counter
#define TINYBVH_IMPLEMENTATION
#include "tiny_bvh.h"
#undef private

using namespace tinybvh;

struct RefScene {
    std::vector<BVH8_CPU*> blas;
    std::vector<BVHBase*> bases;
    std::vector<BLASInstance> inst;
    BVH tlas;
    std::vector<std::vector<bvhvec4>> tris;
};

extern "C" {

void* ref_create(void) { return new RefScene(); }
void ref_destroy(void* s) {
    RefScene* S = (RefScene*)s;
    for (auto b : S->blas) delete b;
    delete S;
}
// triangles: float4 x 3T (Model::triangles, Core/Model.cpp:25-48)
int ref_add_mesh(void* s, int32_t T, const float* tri) {
    RefScene* S = (RefScene*)s;
    S->tris.emplace_back((size_t)T * 3);
    memcpy(S->tris.back().data(), tri, sizeof(float) * 12 * (size_t)T);
    BVH8_CPU* b = new BVH8_CPU();
    b->BuildHQ(S->tris.back().data(), (uint32_t)T);
    S->blas.push_back(b);
    S->bases.push_back(b);
    return (int)S->blas.size() - 1;
}
int ref_add_instance(void* s, int32_t mesh, const float* T16) {
    RefScene* S = (RefScene*)s;
    BLASInstance bi((uint32_t)mesh);
    memcpy(bi.transform, T16, sizeof(float) * 16);
    S->inst.push_back(bi);
    return (int)S->inst.size() - 1;
}
int ref_build(void* s) {
    RefScene* S = (RefScene*)s;
    S->tlas.Build(S->inst.data(), (uint32_t)S->inst.size(), S->bases.data(), (uint32_t)S->bases.size());
    return 0;
}

static inline void set_ray(Ray& r, const float* O, const float* D, const float* rD, float t) {
    memset(&r, 0, sizeof(Ray));
    r.O = bvhvec3(O[0], O[1], O[2]);
    r.D = bvhvec3(D[0], D[1], D[2]);
    r.rD = bvhvec3(rD[0], rD[1], rD[2]);
    r.hit.t = t;
}

// orc_backend-compatible callbacks (oracle/prt_oracle.h)
void ref_closest(void* s, const float* O, const float* D, const float* rD, float* t, float* u, float* v,
                 uint32_t* prim, uint32_t* inst) {
    RefScene* S = (RefScene*)s;
    Ray r; set_ray(r, O, D, rD, *t);
    S->tlas.Intersect(r);
    if (r.hit.t < *t) { *t = r.hit.t; *u = r.hit.u; *v = r.hit.v; *prim = r.hit.prim; *inst = r.hit.inst; }
}
int ref_anyhit(void* s, const float* O, const float* D, const float* rD, float tmax) {
    RefScene* S = (RefScene*)s;
    Ray r; set_ray(r, O, D, rD, tmax);
    return S->tlas.IsOccluded(r) ? 1 : 0;
}

// batch entry points: rays given as (origin, direction) and built with the tinybvh::Ray ctor
// (normalises D, rD = safercp(D), Core/tiny_bvh.h:578-584)
void ref_intersect(void* s, int32_t n, const float* O, const float* D, const float* tmax, float* t, float* u,
                   float* v, uint32_t* prim, uint32_t* inst) {
    RefScene* S = (RefScene*)s;
    for (int i = 0; i < n; i++) {
        Ray r(bvhvec3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), bvhvec3(D[3 * i], D[3 * i + 1], D[3 * i + 2]),
              tmax ? tmax[i] : BVH_FAR);
        S->tlas.Intersect(r);
        t[i] = r.hit.t; u[i] = r.hit.u; v[i] = r.hit.v; prim[i] = r.hit.prim; inst[i] = r.hit.inst;
    }
}
void ref_occluded(void* s, int32_t n, const float* O, const float* D, const float* tmax, int32_t* occ) {
    RefScene* S = (RefScene*)s;
    for (int i = 0; i < n; i++) {
        Ray r(bvhvec3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), bvhvec3(D[3 * i], D[3 * i + 1], D[3 * i + 2]), tmax[i]);
        occ[i] = S->tlas.IsOccluded(r) ? 1 : 0;
    }
}

// Scalar re-walk of BVH8_CPU::Intersect<posX,posY,posZ> (Core/tiny_bvh.h:6313-6474) for one BLAS,
// counting interior (N_int) and leaf (N_leaf) visits.  Returns steps (== library's return value).
static int32_t walk_count(const BVH8_CPU* b, Ray& ray, uint64_t* nint, uint64_t* nleaf) {
    const bool px = ray.D.x > 0, py = ray.D.y > 0, pz = ray.D.z > 0;
    const uint32_t shift = (px ? 3 : 0) + (py ? 6 : 0) + (pz ? 12 : 0);
    uint32_t nodeStack[64]; float distStack[64];
    uint32_t sp = 0, nodeIdx = 0; int32_t steps = 0;
    float tcur = ray.hit.t;
    while (1) {
        steps++;
        if (!(nodeIdx >> 31)) {
            (*nint)++;
            const BVH8_CPU::BVHNode& n = b->bvh8Node[nodeIdx];
            const float* xmin = (const float*)&n.xmin8; const float* xmax = (const float*)&n.xmax8;
            const float* ymin = (const float*)&n.ymin8; const float* ymax = (const float*)&n.ymax8;
            const float* zmin = (const float*)&n.zmin8; const float* zmax = (const float*)&n.zmax8;
            const uint32_t* c8 = (const uint32_t*)&n.child8; const uint32_t* p8 = (const uint32_t*)&n.perm8;
            float tmin[8], tmax[8];
            for (int i = 0; i < 8; i++) {
                float tx1 = ((px ? xmin[i] : xmax[i]) - ray.O.x) * ray.rD.x, tx2 = ((px ? xmax[i] : xmin[i]) - ray.O.x) * ray.rD.x;
                float ty1 = ((py ? ymin[i] : ymax[i]) - ray.O.y) * ray.rD.y, ty2 = ((py ? ymax[i] : ymin[i]) - ray.O.y) * ray.rD.y;
                float tz1 = ((pz ? zmin[i] : zmax[i]) - ray.O.z) * ray.rD.z, tz2 = ((pz ? zmax[i] : zmin[i]) - ray.O.z) * ray.rD.z;
                // _mm256_max_ps(x, y) = x > y ? x : y ; _mm256_min_ps(x, y) = x < y ? x : y
                float a = 0.0f > tx1 ? 0.0f : tx1; a = a > ty1 ? a : ty1; a = a > tz1 ? a : tz1;
                float c = tx2 < tcur ? tx2 : tcur; c = c < ty2 ? c : ty2; c = c < tz2 ? c : tz2;
                tmin[i] = a; tmax[i] = c;
            }
            // permute by octant, then compact valid lanes in order (idxLUT), push ascending lanes
            uint32_t child[8]; float dist[8]; int cnt = 0;
            for (int l = 0; l < 8; l++) {
                uint32_t src = (p8[l] >> shift) & 7;
                int32_t ti, ta; memcpy(&ti, &tmin[src], 4); memcpy(&ta, &tmax[src], 4);
                if (!(ti > ta)) { child[cnt] = c8[src]; dist[cnt] = tmin[src]; cnt++; }
            }
            for (int i = 0; i < cnt; i++) { nodeStack[sp + i] = child[i]; distStack[sp + i] = dist[i]; }
            sp += cnt;
        } else {
            (*nleaf)++;
            const BVHTri4Leaf& leaf = b->bvh8Leaf[nodeIdx & 0x1fffffff];
            float best = 1e30f; int lane = -1;
            float tl[4], ul[4], vl[4]; int ok[4];
            for (int l = 0; l < 4; l++) {
                const float* e2x = (const float*)&leaf.e2x4; const float* e2y = (const float*)&leaf.e2y4; const float* e2z = (const float*)&leaf.e2z4;
                const float* e1x = (const float*)&leaf.e1x4; const float* e1y = (const float*)&leaf.e1y4; const float* e1z = (const float*)&leaf.e1z4;
                const float* v0x = (const float*)&leaf.v0x4; const float* v0y = (const float*)&leaf.v0y4; const float* v0z = (const float*)&leaf.v0z4;
                float hx = ray.D.y * e2z[l] - ray.D.z * e2y[l], hy = ray.D.z * e2x[l] - ray.D.x * e2z[l], hz = ray.D.x * e2y[l] - ray.D.y * e2x[l];
                float sx = ray.O.x - v0x[l], sy = ray.O.y - v0y[l], sz = ray.O.z - v0z[l];
                float det = e1x[l] * hx + e1y[l] * hy + e1z[l] * hz;
                bool m1 = det <= -0.000001f || det >= 0.000001f;
                float id = 1.0f / det;
                float u = (sx * hx + sy * hy + sz * hz) * id;
                float qz = sx * e1y[l] - sy * e1x[l], qx = sy * e1z[l] - sz * e1y[l], qy = sz * e1x[l] - sx * e1z[l];
                float v = (ray.D.x * qx + ray.D.y * qy + ray.D.z * qz) * id;
                float t = (e2x[l] * qx + e2y[l] * qy + e2z[l] * qz) * id;
                ok[l] = m1 && u >= 0 && u <= 1 && v >= 0 && u + v <= 1 && t > 0;
                tl[l] = t; ul[l] = u; vl[l] = v;
            }
            for (int l = 0; l < 4; l++) if (ok[l] && tl[l] <= best) { best = tl[l]; }
            for (int l = 3; l >= 0; l--) if (ok[l] && tl[l] == best) { lane = l; break; }  // __bfind: highest lane
            if (lane >= 0 && best < tcur) {
                tcur = best;
                ray.hit.t = best; ray.hit.u = ul[lane]; ray.hit.v = vl[lane]; ray.hit.prim = leaf.primIdx[lane];
                uint32_t out = 0;
                for (uint32_t i = 0; i < sp; i++) if (distStack[i] < tcur) { nodeStack[out] = nodeStack[i]; distStack[out] = distStack[i]; out++; }
                sp = out;
            }
        }
        if (!sp) break;
        nodeIdx = nodeStack[--sp];
    }
    return steps;
}

// Scalar re-walk of BVH8_CPU::IsOccluded<posX,posY,posZ> (Core/tiny_bvh.h:6488-6601): no octant
// permutation, valid children pushed in lane order, early exit on the first t < tmax.
static bool walk_count_any(const BVH8_CPU* b, const Ray& ray, uint64_t* nint, uint64_t* nleaf) {
    uint32_t nodeStack[128];
    uint32_t sp = 0, nodeIdx = 0;
    const float tcur = ray.hit.t;
    const bool px = ray.D.x > 0, py = ray.D.y > 0, pz = ray.D.z > 0;
    while (1) {
        if (!(nodeIdx >> 31)) {
            (*nint)++;
            const BVH8_CPU::BVHNode& n = b->bvh8Node[nodeIdx];
            const float* xmin = (const float*)&n.xmin8; const float* xmax = (const float*)&n.xmax8;
            const float* ymin = (const float*)&n.ymin8; const float* ymax = (const float*)&n.ymax8;
            const float* zmin = (const float*)&n.zmin8; const float* zmax = (const float*)&n.zmax8;
            const uint32_t* c8 = (const uint32_t*)&n.child8;
            for (int i = 0; i < 8; i++) {
                float tx1 = ((px ? xmin[i] : xmax[i]) - ray.O.x) * ray.rD.x, tx2 = ((px ? xmax[i] : xmin[i]) - ray.O.x) * ray.rD.x;
                float ty1 = ((py ? ymin[i] : ymax[i]) - ray.O.y) * ray.rD.y, ty2 = ((py ? ymax[i] : ymin[i]) - ray.O.y) * ray.rD.y;
                float tz1 = ((pz ? zmin[i] : zmax[i]) - ray.O.z) * ray.rD.z, tz2 = ((pz ? zmax[i] : zmin[i]) - ray.O.z) * ray.rD.z;
                float a = 0.0f > tx1 ? 0.0f : tx1; a = a > ty1 ? a : ty1; a = a > tz1 ? a : tz1;
                float c = tx2 < tcur ? tx2 : tcur; c = c < ty2 ? c : ty2; c = c < tz2 ? c : tz2;
                int32_t ti, ta; memcpy(&ti, &a, 4); memcpy(&ta, &c, 4);
                if (!(ti > ta)) nodeStack[sp++] = c8[i];
            }
        } else {
            (*nleaf)++;
            const BVHTri4Leaf& leaf = b->bvh8Leaf[nodeIdx & 0x1fffffff];
            for (int l = 0; l < 4; l++) {
                const float* e2x = (const float*)&leaf.e2x4; const float* e2y = (const float*)&leaf.e2y4; const float* e2z = (const float*)&leaf.e2z4;
                const float* e1x = (const float*)&leaf.e1x4; const float* e1y = (const float*)&leaf.e1y4; const float* e1z = (const float*)&leaf.e1z4;
                const float* v0x = (const float*)&leaf.v0x4; const float* v0y = (const float*)&leaf.v0y4; const float* v0z = (const float*)&leaf.v0z4;
                float hx = ray.D.y * e2z[l] - ray.D.z * e2y[l], hy = ray.D.z * e2x[l] - ray.D.x * e2z[l], hz = ray.D.x * e2y[l] - ray.D.y * e2x[l];
                float sx = ray.O.x - v0x[l], sy = ray.O.y - v0y[l], sz = ray.O.z - v0z[l];
                float det = e1x[l] * hx + e1y[l] * hy + e1z[l] * hz;
                bool m1 = det <= -0.000001f || det >= 0.000001f;
                float id = 1.0f / det;
                float u = (sx * hx + sy * hy + sz * hz) * id;
                float qz = sx * e1y[l] - sy * e1x[l], qx = sy * e1z[l] - sz * e1y[l], qy = sz * e1x[l] - sx * e1z[l];
                float v = (ray.D.x * qx + ray.D.y * qy + ray.D.z * qz) * id;
                float t = (e2x[l] * qx + e2y[l] * qy + e2z[l] * qz) * id;
                if (m1 && u >= 0 && u <= 1 && v >= 0 && u + v <= 1 && t > 0 && t < tcur) return true;
            }
        }
        if (!sp) break;
        nodeIdx = nodeStack[--sp];
    }
    return false;
}

// Any-hit visit counts for a batch (single-instance scenes); occ_walk/occ_lib per ray for validation.
int ref_count_visits_any(void* s, int32_t n, const float* O, const float* D, const float* tmax, int32_t* occ_walk,
                         int32_t* occ_lib, uint64_t* nint, uint64_t* nleaf) {
    RefScene* S = (RefScene*)s;
    if (S->inst.size() != 1) return -1;
    const BLASInstance& bi = S->inst[0];
    const BVH8_CPU* b = S->blas[bi.blasIdx];
    for (int i = 0; i < n; i++) {
        Ray r;
        memset(&r, 0, sizeof(Ray));
        r.O = bvhvec3(O[3 * i], O[3 * i + 1], O[3 * i + 2]);
        r.D = bvhvec3(D[3 * i], D[3 * i + 1], D[3 * i + 2]);
        r.rD = tinybvh_safercp(r.D);
        r.hit.t = tmax[i];
        Ray tmp = r;
        tmp.O = tinybvh_transform_point(r.O, bi.invTransform);
        tmp.D = tinybvh_transform_vector(r.D, bi.invTransform);
        tmp.rD = tinybvh_safercp(tmp.D);
        occ_walk[i] = walk_count_any(b, tmp, nint, nleaf) ? 1 : 0;
        occ_lib[i] = b->IsOccluded(tmp) ? 1 : 0;
    }
    return 0;
}

// Count visits for a batch of world-space rays through the TLAS (single-instance scenes:
// the TLAS root is a leaf, Core/tiny_bvh.h:1901-1902, so N_tlas = 1, N_inst = 1 per ray).
// out: per-ray steps (re-walk), per-ray library steps, totals of N_int / N_leaf.
int ref_count_visits(void* s, int32_t n, const float* O, const float* D, const float* tmax, int32_t* steps_walk,
                     int32_t* steps_lib, uint64_t* nint, uint64_t* nleaf, float* t_walk) {
    RefScene* S = (RefScene*)s;
    if (S->inst.size() != 1) return -1;
    const BLASInstance& bi = S->inst[0];
    const BVH8_CPU* b = S->blas[bi.blasIdx];
    for (int i = 0; i < n; i++) {
        Ray r(bvhvec3(O[3 * i], O[3 * i + 1], O[3 * i + 2]), bvhvec3(D[3 * i], D[3 * i + 1], D[3 * i + 2]),
              tmax ? tmax[i] : BVH_FAR);
        Ray tmp = r;
        tmp.O = tinybvh_transform_point(r.O, bi.invTransform);
        tmp.D = tinybvh_transform_vector(r.D, bi.invTransform);
        tmp.rD = tinybvh_safercp(tmp.D);
        Ray tmp2 = tmp;
        steps_walk[i] = walk_count(b, tmp, nint, nleaf);
        steps_lib[i] = b->Intersect(tmp2);
        t_walk[i] = tmp.hit.t;
    }
    return 0;
}

}  // extern "C"
