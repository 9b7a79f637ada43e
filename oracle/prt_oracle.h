/*
 * oracle/prt_oracle.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Plain-C restatement of the reference CPU path tracer's hot path
 * (Iancic/Physically-Based-Ray-Tracer @ 2025-08-15):
 *   Renderer::Tick pixel loop        Core/Renderer.cpp:43-141
 *   Renderer::Trace                  Core/Renderer.cpp:150-406
 *   Scene hit-attribute queries      Core/Scene.cpp:41-263
 *   Camera::GetPrimaryRay/SampleSkybox Core/Camera.cpp:29-36,43-74,113-139
 *   BRDF (GGX/Lambert)               Core/BRDF.cpp:16-534, Core/BRDF.h:25-80
 *   tinybvh Ray / MT leaf test       Core/tiny_bvh.h:341,404-422,575-586,6412-6440,6579-6594
 *   RNG (xorshift32, WangHash)       template/tmpl8math.cpp:15-48
 *   RGBF32_to_RGB8                   template/precomp.h:300-316
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline.
 *
 * Parity pinning: the geometric part (closest-hit / any-hit records) is pinned
 * against the reference's own tinybvh v1.4.2 (BVH8_CPU::BuildHQ + TLAS
 * traversal) compiled unmodified from /root/reference into oracle/_ref/
 * (see oracle/Makefile, tests/test_oracle.py).  The shading part
 * (BRDF.cpp, Renderer.cpp, Scene.cpp, Camera.cpp) cannot be compiled here
 * (they need the reference's precomp.h -> windows.h / GLFW / Bullet / assimp),
 * so shading parity is "parity unpinned" against reference binaries: it is a
 * line-by-line restatement with file:line citations and hand-derived
 * known-answer checks (tests/test_oracle.py).
 */
#ifndef PRT_ORACLE_H
#define PRT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* render flags: mirror the public Renderer bools, Core/Renderer.h:33-48 */
#define ORC_AA          (1u << 0)
#define ORC_ACCUMULATE  (1u << 1)
#define ORC_GAMMA       (1u << 2)
#define ORC_NORMALMAP   (1u << 3)
#define ORC_SKYBOX      (1u << 4)
#define ORC_LIGHTED     (1u << 5)
#define ORC_STOCHASTIC  (1u << 6)

/* Renderer::RENDER_STATES, Core/Renderer.h:37-46 */
enum { ORC_MODE_BRDF = 0, ORC_MODE_BASECOLOR, ORC_MODE_GEOMETRYNORMAL, ORC_MODE_SHADINGNORMAL,
       ORC_MODE_METAL, ORC_MODE_ROUGHNESS, ORC_MODE_EMISSIVE };

typedef struct orc_scene orc_scene;

/* post-processing: Renderer::isPostProcessed + Camera::{abberationIntensity, fov, distortion,
 * vignetteIntensity, vignetteRadius, colorGrading} and the camera basis right|up|ahead (9 floats) */
void orc_set_postfx(orc_scene* s, int32_t enabled, int32_t aberration, float fov, float distortion, float vig_int,
                    float vig_rad, const float* grade4, const float* basis9);
void orc_camera_basis(const float* pos3, const float* target3, float* basis9);

typedef struct {
    int32_t width, height;
    int32_t spp;          /* camera paths per pixel in this call (AA: 2 per reference frame) */
    int32_t bounces;      /* Renderer::bounces */
    uint32_t flags;
    int32_t render_mode;
    uint32_t frame_index; /* first reference frame index (RNG stream) */
    uint32_t seed;        /* added to the per-pixel seed base */
} orc_params;

typedef struct {
    uint64_t segments;    /* closest-hit (TLAS) queries */
    uint64_t shadow_rays; /* any-hit (IsOccluded) queries */
    uint64_t paths;
} orc_stats;

/* traversal backend hook: lets the same restated Trace run on tinybvh (oracle/_ref) */
typedef struct {
    void* user;
    /* O, D, rD: ray as tinybvh::Ray holds it (D already normalised). in/out: *t (tmax) */
    void (*closest)(void* user, const float* O, const float* D, const float* rD,
                    float* t, float* u, float* v, uint32_t* prim, uint32_t* inst);
    int (*anyhit)(void* user, const float* O, const float* D, const float* rD, float tmax);
} orc_backend;

/* extensions: instance material kinds (the reference's dead Scene.cpp:193-205 branches)
 * and one area light (never sampled by the reference's Trace) */
#define ORC_MAT_TEXTURED   0
#define ORC_MAT_DIELECTRIC 1
#define ORC_MAT_MIRROR     2
int orc_set_instance_material(orc_scene* s, int32_t inst, int32_t kind);
void orc_set_area_light(orc_scene* s, int32_t enabled, const float* corner3, const float* edge_u3, const float* edge_v3,
                        const float* radiance3, int32_t two_sided);

orc_scene* orc_scene_create(void);
void orc_scene_destroy(orc_scene* s);
int orc_add_texture(orc_scene* s, int32_t w, int32_t h, const uint32_t* pixels);
int orc_add_mesh(orc_scene* s, int32_t tri_count, const float* triangles /*12T*/, const float* fixed_normals /*12T*/,
                 const float* fixed_uvs /*6T*/, const int32_t* indices /*3T*/, const float* vertices /*3V*/,
                 int32_t vertex_count, const float* face_normals /*3T*/,
                 int32_t albedo, int32_t normal, int32_t metalness, int32_t emission);
int orc_add_instance(orc_scene* s, int32_t mesh, const float* transform16);
void orc_set_lights(orc_scene* s, const float* point_pos12, const float* point_col12, const float* dir_pos3,
                    const float* dir_col3, const float* spot_pos3, const float* spot_col3, const float* spot_rot3);
void orc_set_sky(orc_scene* s, int32_t w, int32_t h, const float* rgb);
void orc_set_camera(orc_scene* s, const float* pos3, const float* tl3, const float* tr3, const float* bl3);
int orc_build(orc_scene* s);
void orc_set_backend(orc_scene* s, const orc_backend* b); /* NULL -> built-in BVH */

/* camera basis from position/target, Core/Camera.cpp:29-36 */
void orc_camera_lookat(const float* pos3, const float* target3, float aspect, float* tl3, float* tr3, float* bl3);

/* Renderer::Tick semantics over (spp / paths-per-frame) reference frames.
 * acc (float4 W*H), nsamp (int W*H), dist (float W*H) is the persistent
 * accumulation state (Core/Renderer.h:61-63).  avg_rgba / rgb8 may be NULL. */
int orc_render(orc_scene* s, const orc_params* p, float* acc, int32_t* nsamp, float* dist,
               float* avg_rgba, uint32_t* rgb8, int32_t nthreads, orc_stats* stats);

/* per-frame raw values (after AA average + gamma, before accumulation): out float4 [frames][W*H], t1 [frames][W*H] */
int orc_render_frames(orc_scene* s, const orc_params* p, float* frame_rgba, float* t_primary,
                      int32_t nthreads, orc_stats* stats);

/* geometry-only queries */
int orc_primary_hits(orc_scene* s, int32_t w, int32_t h, float* t, float* u, float* v, uint32_t* prim, uint32_t* inst,
                     int32_t nthreads);
int orc_intersect(orc_scene* s, int32_t n, const float* origins, const float* dirs, const float* tmax,
                  float* t, float* u, float* v, uint32_t* prim, uint32_t* inst, int32_t nthreads);
int orc_occluded(orc_scene* s, int32_t n, const float* origins, const float* dirs, const float* tmax,
                 int32_t* occluded, int32_t nthreads);

/* rays Trace fires for every stride-th pixel (7 floats each: O, D, tmax); single-threaded */
int orc_collect_rays(orc_scene* s, const orc_params* p, int32_t stride, float* closest, int64_t cap_closest,
                     float* anyhit, int64_t cap_any, int64_t* n_closest, int64_t* n_any);

/* function-level entry points for unit tests */
uint32_t orc_init_seed(uint32_t base);
void orc_rng_floats(uint32_t seed, int32_t n, float* out);
void orc_eval_combined_brdf(const float* N, const float* L, const float* V, const float* mat8, float* out3);
float orc_brdf_probability(const float* mat8, const float* V, const float* N);
int orc_brdf_probe(int32_t op, int32_t n, const float* in, float* out);  /* include/prt.h prt_brdf_probe records */
int orc_eval_indirect(const float* u2, const float* N, const float* V, const float* mat8, int32_t type,
                      float* dir3, float* weight3);
void orc_sample_sky(orc_scene* s, const float* D, float* out3);
uint32_t orc_pack_rgb8(const float* rgba);

#ifdef __cplusplus
}
#endif
#endif
