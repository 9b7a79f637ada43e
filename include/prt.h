/*
 * prt.h -- C ABI of the MI355X-native path-tracing hot path.
 *
 * Drop-in boundary for the reference's per-pixel hot path (Iancic/Physically-Based-Ray-Tracer):
 * a Renderer::Tick shim replaces Core/Renderer.cpp:43-141 with prt_render(),
 * after handing over the data the hot path reads without copying:
 *
 *   prt_set_textures   <- Model::{albedo,normal,metalness,emission}Texture (template/surface.h:49-94)
 *   prt_set_meshes     <- Model fat-triangle arrays (Core/Model.h:36-44, Core/Model.cpp:25-119)
 *   prt_set_instances  <- Scene::blases[i].transform + gameobjects[i]->modelIndex (Core/Scene.cpp:220-223,
 *                         Core/tiny_bvh.h:1243-1256)
 *   prt_set_lights     <- Renderer point-light SoA (Core/Renderer.h:80-88), directionalLights[0], spotlights[0]
 *   prt_set_sky        <- Camera::skyPixels (Core/Camera.cpp:9)
 *   prt_set_camera     <- Camera::camPos/topLeft/topRight/bottomLeft/right/up/ahead (Core/Camera.cpp:29-36)
 *   prt_set_postfx     <- Renderer::isPostProcessed + Camera post-process members (Core/Camera.h:11-31)
 *   prt_render         <- the OpenMP pixel loop + Renderer::Trace (Core/Renderer.cpp:43-141,150-406)
 *
 * Conventions: plain pointers and sizes, no C++ types; every call returns PRT_OK (0) or a negative
 * prt_status; prt_last_error() gives the message for the calling thread.  No exceptions cross the ABI.
 * One host thread per context.  All scene arrays are copied to device memory (HBM) during the call;
 * the caller may free them afterwards.  A HIP device must be present: there is no CPU fallback.
 * Ordering: prt_set_textures / prt_set_meshes / prt_set_sky first wait for the frames queued on the
 * context's stream (they overwrite resident buffers); prt_set_instances / prt_set_instance_materials are
 * stream-ordered (a frame queued before the call renders the old instances); the remaining setters are
 * read at the next prt_render.
 */
#ifndef PRT_H
#define PRT_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRT_ABI_VERSION 10

typedef enum {
    PRT_OK = 0,
    PRT_ERR_INVALID_ARGUMENT = -1,
    PRT_ERR_NO_DEVICE = -2,
    PRT_ERR_HIP = -3,
    PRT_ERR_OUT_OF_MEMORY = -4,
    PRT_ERR_NOT_READY = -5,     /* scene/camera incomplete */
    PRT_ERR_UNSUPPORTED = -6
} prt_status;

/* Render flags: the public Renderer bools, Core/Renderer.h:33,48 */
#define PRT_FLAG_AA          (1u << 0)
#define PRT_FLAG_ACCUMULATE  (1u << 1)
#define PRT_FLAG_GAMMA       (1u << 2)
#define PRT_FLAG_NORMALMAP   (1u << 3)
#define PRT_FLAG_SKYBOX      (1u << 4)
#define PRT_FLAG_LIGHTED     (1u << 5)
#define PRT_FLAG_STOCHASTIC  (1u << 6)
/* the reference's defaults (Core/Renderer.h:33,48) */
#define PRT_FLAGS_DEFAULT    (0x7Fu)

/* Renderer::RENDER_STATES, Core/Renderer.h:37-46 */
typedef enum {
    PRT_MODE_BRDF = 0, PRT_MODE_BASECOLOR = 1, PRT_MODE_GEOMETRYNORMAL = 2, PRT_MODE_SHADINGNORMAL = 3,
    PRT_MODE_METAL = 4, PRT_MODE_ROUGHNESS = 5, PRT_MODE_EMISSIVE = 6
} prt_render_mode;

typedef struct prt_ctx prt_ctx;

typedef struct {
    int32_t device;      /* HIP device ordinal (one process per GPU) */
    uint32_t flags;      /* reserved, 0 */
} prt_device_desc;

/* one packed 0x00RRGGBB texture, exactly Surface::pixels (template/surface.cpp:47-66) */
typedef struct {
    int32_t width, height;
    const uint32_t* pixels;
} prt_texture;

/* one Model (Core/Model.h:36-44).  T = tri_count, V = vertex_count. */
typedef struct {
    int32_t tri_count;
    int32_t vertex_count;
    const float* triangles;      /* float4 x 3T : Model::triangles (fat, w ignored)            */
    const float* fixed_normals;  /* float4 x 3T : Model::fixedNormals                          */
    const float* fixed_uvs;      /* float2 x 3T : Model::fixedTextureCoords                    */
    const int32_t* indices;      /* int x 3T    : Model::indices                               */
    const float* vertices;       /* float3 x V  : Model::vertices                              */
    const float* face_normals;   /* float3 x T  : Model::faceNormals                           */
    int32_t albedo_tex;          /* required (Core/Scene.cpp:160 dereferences it)              */
    int32_t normal_tex;          /* -1 = none */
    int32_t metalness_tex;       /* -1 = none (G = roughness, B = metalness, Scene.cpp:175-181) */
    int32_t emission_tex;        /* -1 = none */
} prt_mesh;

/* lights as the hot path reads them (Core/Renderer.cpp:216-310) */
typedef struct {
    float point_pos[4][3];   /* posX/posY/posZ SoA of the 4 SIMD point lights */
    float point_color[4][3];
    float dir_pos[3], dir_color[3];                  /* directionalLights[0]->transform */
    float spot_pos[3], spot_color[3], spot_rot[3];   /* spotlights[0]->transform        */
} prt_lights;

/* Instance material kinds (prt_set_instance_materials).  The reference's Scene::GetMaterialBRDF has a
 * dielectric and a perfect-mirror branch gated on `modelIndex == -1`, which never holds (Core/Scene.cpp:
 * 193-205, "Instead of -1 place model index"); here the caller names the instances that take them.
 * DIELECTRIC takes Renderer::Trace's glass branch (Core/Renderer.cpp:331-372: reflection + refraction
 * rays, Schlick-weighted, depth first); MIRROR forces metalness 1 / roughness 0 (the :376 fast path). */
#define PRT_MAT_TEXTURED   0
#define PRT_MAT_DIELECTRIC 1
#define PRT_MAT_MIRROR     2

/* One emitting parallelogram corner + a*edge_u + b*edge_v (a, b in [0,1]) -- an extension: the reference's
 * AreaLight (Core/AreaLight.h) is never sampled by Trace.  Radiance on the side of cross(edge_u, edge_v)
 * (both sides when two_sided); sampled by next-event estimation at every lit hit and reached by BRDF rays,
 * combined with the power heuristic. */
typedef struct {
    float corner[3], edge_u[3], edge_v[3];
    float radiance[3];
    int32_t two_sided;
} prt_area_light;

/* Camera screen plane and basis (Core/Camera.cpp:29-36, 113-139; Core/Camera.h:15-17).  right / up /
 * ahead are only read by the Panini projection (post-processing on); prt_camera_look_at fills all. */
typedef struct {
    float pos[3];
    float top_left[3], top_right[3], bottom_left[3];
    float right[3], up[3], ahead[3];
} prt_camera;

typedef struct {
    int32_t width, height;
    int32_t spp;            /* camera paths per pixel in this call; with AA one reference frame = 2 paths */
    int32_t bounces;        /* Renderer::bounces (closest-hit segments per path), 0..16 */
    uint32_t flags;         /* PRT_FLAG_* */
    int32_t render_mode;    /* prt_render_mode */
    uint32_t frame_index;   /* first reference frame of this call (RNG stream) */
    uint32_t seed;          /* added to the per-pixel seed base */
} prt_render_params;

typedef struct {
    uint64_t segments;      /* closest-hit queries (TLAS intersections) */
    uint64_t shadow_rays;   /* any-hit queries (IsOccluded) */
    uint64_t paths;         /* camera paths traced */
    double   ms;            /* device time of the render (HIP events) */
    double   ms_trace;      /* device time of the path-tracing kernel(s) only */
    double   ms_closest;    /* device time of the traversal launches (closest + shadow rays together), summed */
    double   ms_anyhit;     /* reserved (0): shadow rays are traced inside the merged traversal launches */
    int32_t  pipeline;      /* 2 = the merged-trace wavefront (prt_wave2.hip) */
    int32_t  iterations;    /* traversal launches per call */
    int32_t  batches;       /* 1 */
    int32_t  ranks;         /* shards whose rays these stats count (1 unless a local group summed its members) */
    uint64_t stack_overflows; /* traversal stack overflows since the context was created: a BVH node group that
                                 found no free stack level (the host sizes the stacks from the BVH depth, so any
                                 non-zero count is a builder / sizing bug; the results may have lost hits) */
} prt_stats;

/* closest-hit record, tinybvh::Intersection (Core/tiny_bvh.h:545-567) minus user data */
typedef struct {
    float t, u, v;
    uint32_t prim, inst;
} prt_hit;

/* ---- context ---- */
int prt_abi_version(void);
const char* prt_last_error(void);
int prt_device_count(int32_t* count);
int prt_create(const prt_device_desc* desc, prt_ctx** out);
int prt_destroy(prt_ctx* ctx);
/* run subsequent work on an external hipStream_t (e.g. torch's current stream); NULL = ctx-owned stream */
int prt_set_stream(prt_ctx* ctx, void* hip_stream);
/* Frames in flight (ABI 9; the reference's Renderer::Tick renders one frame per call, Core/Renderer.cpp:43-141).
 * n = 1 (default): a prt_render call's work is complete in the context stream's order when the call returns.
 * n = 2..8 (ABI 10; 2..4 in ABI 9): a prt_render with device outputs (or a prt_render_tiles) and no stats enqueues its frame on one of n
 * internal streams, forked from the context stream, so its wavefront chain overlaps those of the previous n - 1
 * calls; the accumulation (and a sharded frame's gather and untile) still run in call order, so the results are
 * bit-identical to n = 1.  A call's outputs are complete in the context stream's order once n - 1 more render
 * calls have been enqueued, or after prt_finish.  prt_set_instances / prt_set_instance_materials (ABI 10) do not
 * join them: the instance state has n + 1 device copies and an update writes the next one once the frames that
 * read it are done (a stream wait).  Every other entry point (and a render with host outputs or stats) joins the
 * frames in flight first.  Local shard groups: n = 1 only (PRT_ERR_UNSUPPORTED). */
int prt_set_frames_in_flight(prt_ctx* ctx, int32_t n);
/* the context stream waits for every frame in flight (no host wait) */
int prt_finish(prt_ctx* ctx);

/* ---- scene (Scene / Model / Camera state) ---- */
int prt_set_textures(prt_ctx* ctx, const prt_texture* textures, int32_t count);
int prt_set_meshes(prt_ctx* ctx, const prt_mesh* meshes, int32_t count);
/* transforms: 16*count floats, row-major BLASInstance::transform; mesh_index: count.  Above 64 instances the rays
 * walk an instance BVH, rebuilt for every call as the reference's per-frame BVH::Build (a host SAH build): on the
 * calling thread when the instance count changes, otherwise on the context's worker thread, the context stream
 * waiting for that build before its upload (the caller neither builds nor waits) */
int prt_set_instances(prt_ctx* ctx, const float* transforms, const uint32_t* mesh_index, int32_t count);
int prt_set_lights(prt_ctx* ctx, const prt_lights* lights);
/* kinds: one PRT_MAT_* per instance (count = the instance count), or count 0 = all textured.  Reset by
 * prt_set_instances with a different instance count.  Dielectric instances need bounces <= 4 with AA (5 without): the depth-first path tree
 * has up to 2^bounces - 1 segments per path. */
int prt_set_instance_materials(prt_ctx* ctx, const int32_t* kinds, int32_t count);
/* count 0 (none) or 1 */
int prt_set_area_lights(prt_ctx* ctx, const prt_area_light* lights, int32_t count);
/* float RGB equirect, w*h*3; NULL/0 = no sky (misses shade 0 even with PRT_FLAG_SKYBOX) */
int prt_set_sky(prt_ctx* ctx, const float* rgb, int32_t width, int32_t height);
int prt_set_camera(prt_ctx* ctx, const prt_camera* cam);
/* Camera::Camera basis from position/target and aspect (Core/Camera.cpp:29-36) */
int prt_camera_look_at(const float pos[3], const float target[3], float aspect, prt_camera* out);

/* Post-processing (Renderer::isPostProcessed, Core/Renderer.h:48): Panini primary rays
 * (Camera::GetPrimaryRay/Panini, Core/Camera.cpp:81-139) and the screen pass of Core/Renderer.cpp:107-133
 * (chromatic aberration from the accumulator, vignette, colour grading).  avg_rgba stays the plain
 * average; rgb8 gets the post-processed pixel. */
typedef struct {
    int32_t enabled;            /* Renderer::isPostProcessed (default false) */
    int32_t aberration;         /* Camera::abberationIntensity, pixels */
    float fov;                  /* Camera::fov (Camera::Panini uses it as radians, :86) */
    float distortion;           /* Camera::distortion */
    float vignette_intensity;   /* Camera::vignetteIntensity */
    float vignette_radius;      /* Camera::vignetteRadius (the pow exponent) */
    float color_grading[4];     /* Camera::colorGrading */
} prt_postfx;
/* preset 0: the Camera member defaults (Core/Camera.h:12,23,27; DEBUGMODE build), 1: the GAME preset P1
 * (Core/Camera.cpp:18-23, vignetteRadius keeps its default: the constructor self-assigns it).
 * enabled is set to 1. */
int prt_postfx_preset(int32_t preset, prt_postfx* out);
int prt_set_postfx(prt_ctx* ctx, const prt_postfx* pfx);

/* ---- rendering (Renderer::Tick) ----
 * Traces params.spp camera paths per pixel as spp/2 (AA) or spp reference frames and folds each
 * frame into the persistent accumulation state exactly as Core/Renderer.cpp:81-104 does.
 * Outputs (either may be NULL): avg_rgba = float4 W*H average, rgb8 = 0x00RRGGBB W*H.
 * They are host pointers unless PRT_OUT_DEVICE is set in out_flags (then device pointers). */
#define PRT_OUT_DEVICE (1u << 0)
int prt_render(prt_ctx* ctx, const prt_render_params* params, float* avg_rgba, uint32_t* rgb8,
               uint32_t out_flags, prt_stats* stats);
/* Reset the accumulation state: memset of the accumulator (Core/Renderer.cpp:147) and, with
 * full != 0, also samplesPerPixel/distances (fresh Renderer). */
int prt_reset_accumulation(prt_ctx* ctx, int32_t full);
/* Running ray totals (ABI 7): closest-hit segments and shadow rays of every render since the context was created
 * or last reset, counted on the device at the end of each render (the figure behind the reference's ImGui ray
 * counter, Core/Renderer.cpp:467-474) so a frame loop need not pass prt_stats, which waits for each frame.  Waits for
 * the frames queued on the context's stream (a local group: on every member's, summed); reset != 0 zeroes the totals
 * after reading them. */
int prt_ray_totals(prt_ctx* ctx, uint64_t* segments, uint64_t* shadow_rays, int32_t reset);

/* ---- checkpoint / resume of the progressive accumulation (the reference keeps it in memory only) ----
 * The accumulation state Renderer holds between Ticks (Core/Renderer.h:61-63: accumulator, samplesPerPixel,
 * distances) as one opaque blob with a header recording the image and shard geometry it belongs to.
 * prt_accumulation_bytes: the blob size (0 before the first render).  prt_save_accumulation: copies the state
 * out (waits for the frames queued on the context's stream).  prt_load_accumulation: restores it into a context
 * of the same shard geometry; the next prt_render with the same image size continues bit-identically (the caller
 * restores its frame_index too: the RNG stream is keyed by it).  A mismatched or truncated blob:
 * PRT_ERR_INVALID_ARGUMENT; a local group (prt_create_group): PRT_ERR_UNSUPPORTED (one blob per rank's context
 * with RCCL). */
int prt_accumulation_bytes(prt_ctx* ctx, uint64_t* bytes);
int prt_save_accumulation(prt_ctx* ctx, void* blob, uint64_t bytes);
int prt_load_accumulation(prt_ctx* ctx, const void* blob, uint64_t bytes);

/* ---- multi-GPU inside the boundary ----
 * A sharded context renders only its rank's pixel tiles (tile_size x tile_size, numbered row-major, dealt
 * round-robin: rank r owns tiles r, r + world, ...), and prt_render gathers the per-rank tile buffers on
 * rank 0 once per frame, replacing the reference's single-process OpenMP row loop (Core/Renderer.cpp:43).
 * Rank 0's outputs then hold the whole frame; the other ranks' outputs are not written (may be NULL).
 * Stats count the calling rank's rays (a local group sums its members, stats.ranks = world).
 * Post-processing shards except the chromatic aberration (neighbours' accumulators): PRT_ERR_UNSUPPORTED.
 *
 * One process per GPU over RCCL (xGMI): rank 0 makes an id, the caller carries its bytes to the other
 * ranks over any host channel (torch.distributed, MPI, a file), every rank joins with its own context.
 * The context owns the communicator; RCCL is loaded on first use (the copy the process already holds). */
#define PRT_SHARD_ID_BYTES 128
int prt_shard_unique_id(uint8_t id[PRT_SHARD_ID_BYTES]);
int prt_shard_init_rccl(prt_ctx* ctx, const uint8_t id[PRT_SHARD_ID_BYTES], int32_t rank, int32_t world,
                        int32_t tile_size);
/* ... or an existing communicator (ncclComm_t, not owned: the caller destroys it after prt_destroy) */
int prt_shard_attach_rccl(prt_ctx* ctx, void* nccl_comm, int32_t tile_size);
/* One process, several devices (prt_create with a device list).  The group context is member 0;
 * every setter applies to all members, prt_render renders all shards concurrently (one stream per member)
 * and gathers them on member 0 with device-to-device copies.  A device may repeat (several shards on one
 * GPU: how the decomposition is tested on a one-GPU box). */
int prt_create_group(const prt_device_desc* devices, int32_t count, int32_t tile_size, prt_ctx** out);
typedef struct {
    int32_t rank, world, tile_size;
    int32_t transport;      /* 0 = none (whole frame), 1 = RCCL, 2 = local group */
} prt_shard_info;
int prt_get_shard_info(prt_ctx* ctx, prt_shard_info* info);

/* ---- pixel-tile sharding with a caller-side transport (the building blocks of the above) ----
 * The image is cut into tile_size x tile_size tiles numbered in row-major order; rank r renders
 * tiles r, r+world, r+2*world, ...  into a compact float4 buffer laid out
 * [local_tile][tile_size*tile_size] (pixels outside the image are written as 0).
 * prt_tile_buffer_pixels() gives the element count (per rank, equal on all ranks: the max). */
int prt_tile_buffer_pixels(int32_t width, int32_t height, int32_t tile_size, int32_t world, int64_t* pixels);
/* host-only: image pixel index (y*width + x) of every element of rank's tile buffer, -1 where the tile
 * overhangs the image; pixel_of_slot holds prt_tile_buffer_pixels() entries.  No device needed. */
int prt_tile_pixel_map(int32_t width, int32_t height, int32_t tile_size, int32_t rank, int32_t world,
                       int32_t* pixel_of_slot);
int prt_render_tiles(prt_ctx* ctx, const prt_render_params* params, int32_t tile_size, int32_t rank,
                     int32_t world, float* tiles_rgba_device, prt_stats* stats);
/* rank-0 side: gathered [world][tile_buffer_pixels] float4 device buffer -> W*H avg_rgba + rgb8 (device).
 * With post-processing the vignette / grading apply to rgb8; chromatic aberration needs the neighbours'
 * accumulators, which stay on their ranks: PRT_ERR_UNSUPPORTED there. */
int prt_untile(prt_ctx* ctx, const float* gathered_device, int32_t width, int32_t height, int32_t tile_size,
               int32_t world, float* avg_rgba_device, uint32_t* rgb8_device);

/* ---- geometry-only queries (the traversal kernels on their own) ---- */
/* primary-ray closest hits for every pixel (config C2): out = W*H prt_hit (host or device per out_flags) */
int prt_trace_primary(prt_ctx* ctx, int32_t width, int32_t height, prt_hit* hits, uint32_t out_flags,
                      prt_stats* stats);
/* arbitrary rays: origins/dirs float3 x n (dirs normalised like the tinybvh::Ray ctor), tmax n (NULL = 1e30) */
int prt_intersect(prt_ctx* ctx, int32_t n, const float* origins, const float* dirs, const float* tmax,
                  prt_hit* hits);
int prt_occluded(prt_ctx* ctx, int32_t n, const float* origins, const float* dirs, const float* tmax,
                 int32_t* occluded);

/* ---- shading-function probe (ABI 10): the device's own BRDF functions (the ones the shading kernels inline) on
 * n host records, for known-answer tests of the BRDF restatement (Core/BRDF.cpp).  Record k: in[24 k ..], out[8 k ..].
 *   EVAL         BRDF::evalCombinedBRDF (:439-452)     in N[0..2] L[3..5] V[6..8] material[9..16]    out rgb[0..2]
 *   PROBABILITY  BRDF::getBrdfProbability (:504-526)   in N, V, material                          out p[0]
 *   INDIRECT     BRDF::evalIndirectCombinedBRDF (:454-502, weight in = 1)  in N, V, material, u[17..18],
 *                type[19] (1 diffuse, 2 specular)      out ok[0] dir[1..3] weight[4..6]
 *   GGX_D        ggxD (:218-222)                       in alphaSquared[0] NdotH[1]                out D[0]
 *   SMITH_G2     Smith_G2 height-correlated, divided by the denominator (:189-208)
 *                                                      in alphaSquared[0] NdotL[1] NdotV[2]       out G2[0]
 *   FRESNEL      evalFresnel Schlick (:84-87)          in f0[0..2] f90[3] NdotS[4]                out F[0..2]
 *   SHADOWED_F90 shadowedF90 (:100-104)                in F0[0..2]                                out f90[0]
 *   VNDF         sampleGGXVNDF (:224-269)              in Ve[0..2] alphaX[3] alphaY[4] u[5..6]    out H[0..2]
 * material = base rgb, metalness, emissive rgb, roughness (MaterialProperties, Core/BRDF.h:165-176). */
#define PRT_PROBE_EVAL 0
#define PRT_PROBE_PROBABILITY 1
#define PRT_PROBE_INDIRECT 2
#define PRT_PROBE_GGX_D 3
#define PRT_PROBE_SMITH_G2 4
#define PRT_PROBE_FRESNEL 5
#define PRT_PROBE_SHADOWED_F90 6
#define PRT_PROBE_VNDF 7
int prt_brdf_probe(prt_ctx* ctx, int32_t op, int32_t n, const float* in, float* out);

/* ---- BLAS builder (the reference builds on the CPU, Core/tiny_bvh.h:1968-2284,3706-3781)
 * HOST_SAH (default): binned SAH binary tree + SAH-optimal 8-wide collapse on the host.
 * GPU_LBVH: Morton-code LBVH (Karras 2012) + treelet restructuring + SAH-optimal 8-wide collapse on the device,
 * Node8 layout only.
 * Applies to the next prt_set_meshes.  Hits do not depend on the builder (order-independent hit rule). */
#define PRT_BUILDER_HOST_SAH 0
#define PRT_BUILDER_GPU_LBVH 1
#define PRT_BUILDER_HOST_SBVH 2  /* spatial splits (BVH::BuildHQ, Core/tiny_bvh.h:1968-2284) + SAH-optimal collapse */
#define PRT_BUILDER_GPU_PLOC 3   /* device PLOC clustering + SAH-optimal collapse */
int prt_set_bvh_builder(prt_ctx* ctx, int32_t builder);

/* ---- introspection ---- */
typedef struct {
    int64_t blas_nodes;     /* device BVH nodes over all meshes */
    int64_t blas_leaves;
    int64_t device_bytes;   /* BVH + triangle + shading arrays resident in HBM */
    int32_t max_depth;
    int32_t triangles;
    double  build_ms;       /* wall time of the last prt_set_meshes (BLAS builds + uploads) */
    int32_t builder;        /* PRT_BUILDER_* used by the last prt_set_meshes */
    int32_t tlas_depth;     /* levels of the instance BVH the rays walk (0: instances tested as a linear list) */
    int32_t tlas_rebuilds;  /* rebuilds of the instance BVH since the instance count last changed: one per
                               prt_set_instances */
    int32_t tlas_async;     /* (ABI 10) of those, built on the context's worker thread in stream order (every update
                               after the one that set the instance count) */
    int32_t tlas_median;    /* (ABI 10) of the worker's builds, balanced median-split trees: the SAH tree was deeper
                               than the traversal stacks were sized for at the instance count's first build */
    float   tlas_build_ms;     /* (ABI 10) wall time of the worker's last build (instance boxes + build + collapse) */
    float   tlas_build_cpu_ms; /* (ABI 10) its thread CPU time */
} prt_scene_info;
int prt_get_scene_info(prt_ctx* ctx, prt_scene_info* info);

#ifdef __cplusplus
}
#endif
#endif /* PRT_H */
