// prt_renderer.hpp -- C++ host mirror of the reference's Renderer / Scene / Camera API surface
// (Core/Renderer.h:12-112, Core/Scene.h:12-80, Core/Camera.h:11-37, Core/Model.h:36-44) on top of the C ABI
// in prt.h.  Header-only C++17; link libprt.so.  The names and meanings of the public members follow the
// reference so a Renderer::Tick port reads like the original; the hot path (Tick's pixel loop +
// Renderer::Trace, Core/Renderer.cpp:43-141,150-406) runs on the GPU through prt_render().
//
// Differences from the reference, all outside the hot path: the Scene is filled by the caller (the
// reference's assimp / JSON loading, Core/Scene.cpp:10-28,279-340, stays where it is), physics and UI
// are not part of this header, and errors surface as prt::Error exceptions instead of crashes.
#pragma once
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "prt.h"

namespace prt {

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string& what) : std::runtime_error(what), code(code) {}
  int code;
};

inline void check(int rc) {
  if (rc != PRT_OK) throw Error(rc, std::string("prt error ") + std::to_string(rc) + ": " + prt_last_error());
}

// Model (Core/Model.h:36-44): the fat per-corner arrays the hot path reads, owned here.
struct Model {
  std::vector<float> triangles;           // float4 x 3T (Model::triangles)
  std::vector<float> fixedNormals;        // float4 x 3T
  std::vector<float> fixedTextureCoords;  // float2 x 3T
  std::vector<int32_t> indices;           // 3T
  std::vector<float> vertices;            // float3 x V
  std::vector<float> faceNormals;         // float3 x T
  int32_t albedoTexture = -1, normalTexture = -1, metalnessTexture = -1, emissionTexture = -1;  // Scene::textures ids
  int32_t TriCount() const { return (int32_t)(indices.size() / 3); }
};

// Surface (template/surface.h:49-94): packed 0x00RRGGBB pixels
struct Texture {
  int32_t width = 0, height = 0;
  std::vector<uint32_t> pixels;
};

// GameObject + BLASInstance (Core/GameObject.h, Core/tiny_bvh.h:1243-1256): row-major 4x4 and model index
struct GameObject {
  std::array<float, 16> transform{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  uint32_t modelIndex = 0;
  int32_t material = PRT_MAT_TEXTURED;  // the model index Scene.cpp:193-205 should have tested: DIELECTRIC / MIRROR
};

class Scene {
 public:
  std::vector<Model> models;
  std::vector<Texture> textures;
  std::vector<GameObject> gameobjects;
  prt_lights lights{};              // Renderer point-light SoA + directionalLights[0] + spotlights[0]
  std::vector<float> skyPixels;     // Camera::skyPixels, float RGB equirect (empty = no sky)
  int32_t skyWidth = 0, skyHeight = 0;
  std::vector<prt_area_light> areaLights;  // Scene::areaLights (Core/AreaLight.h): at most one, sampled with MIS

  // everything the hot path reads, copied to HBM (Scene::Init + BuildTLAS, Core/Scene.cpp:10-28,220-223)
  void Upload(prt_ctx* ctx) const {
    std::vector<prt_texture> tex;
    for (const Texture& t : textures) tex.push_back({t.width, t.height, t.pixels.data()});
    check(prt_set_textures(ctx, tex.data(), (int32_t)tex.size()));
    std::vector<prt_mesh> ms;
    for (const Model& m : models) {
      prt_mesh d{};
      d.tri_count = m.TriCount();
      d.vertex_count = (int32_t)(m.vertices.size() / 3);
      d.triangles = m.triangles.data();
      d.fixed_normals = m.fixedNormals.data();
      d.fixed_uvs = m.fixedTextureCoords.data();
      d.indices = m.indices.data();
      d.vertices = m.vertices.data();
      d.face_normals = m.faceNormals.data();
      d.albedo_tex = m.albedoTexture;
      d.normal_tex = m.normalTexture;
      d.metalness_tex = m.metalnessTexture;
      d.emission_tex = m.emissionTexture;
      ms.push_back(d);
    }
    check(prt_set_meshes(ctx, ms.data(), (int32_t)ms.size()));
    UploadInstances(ctx);
    check(prt_set_lights(ctx, &lights));
    check(prt_set_area_lights(ctx, areaLights.empty() ? nullptr : areaLights.data(), (int32_t)areaLights.size()));
    check(prt_set_sky(ctx, skyPixels.empty() ? nullptr : skyPixels.data(), skyWidth, skyHeight));
  }
  // GameObject::Synchronise moved an instance: new transforms, TLAS rebuilt (Core/Renderer.cpp:33-41)
  void UploadInstances(prt_ctx* ctx) const {
    std::vector<float> xf;
    std::vector<uint32_t> mi;
    std::vector<int32_t> mat;
    bool any = false;
    for (const GameObject& g : gameobjects) {
      xf.insert(xf.end(), g.transform.begin(), g.transform.end());
      mi.push_back(g.modelIndex);
      mat.push_back(g.material);
      any = any || g.material != PRT_MAT_TEXTURED;
    }
    check(prt_set_instances(ctx, xf.data(), mi.data(), (int32_t)mi.size()));
    check(prt_set_instance_materials(ctx, any ? mat.data() : nullptr, any ? (int32_t)mat.size() : 0));
  }
};

// Camera (Core/Camera.h:11-31): position, target, the screen plane GetPrimaryRay interpolates, its basis
// and the post-process members (defaults of Camera.h; read when Renderer::isPostProcessed is set)
class Camera {
 public:
  float camPos[3] = {0, 0, -1}, camTarget[3] = {0, 0, 0};
  float aspect = 1.0f;
  float topLeft[3] = {}, topRight[3] = {}, bottomLeft[3] = {};
  float right[3] = {}, up[3] = {}, ahead[3] = {};
  float colorGrading[4] = {1.f, 1.f, 1.f, 1.f};
  float fov = 40.f, distortion = 40.f, vignetteIntensity = 20.f, vignetteRadius = 0.3f;
  int32_t abberationIntensity = 0;

  Camera() = default;
  Camera(const float pos[3], const float target[3], float aspect_) : aspect(aspect_) {
    for (int k = 0; k < 3; k++) { camPos[k] = pos[k]; camTarget[k] = target[k]; }
    Update();
  }
  // the basis of Camera::Camera / HandleInput (Core/Camera.cpp:29-36)
  void Update() {
    prt_camera c{};
    check(prt_camera_look_at(camPos, camTarget, aspect, &c));
    for (int k = 0; k < 3; k++) {
      topLeft[k] = c.top_left[k]; topRight[k] = c.top_right[k]; bottomLeft[k] = c.bottom_left[k];
      right[k] = c.right[k]; up[k] = c.up[k]; ahead[k] = c.ahead[k];
    }
  }
  prt_camera Plane() const {
    prt_camera c{};
    for (int k = 0; k < 3; k++) {
      c.pos[k] = camPos[k]; c.top_left[k] = topLeft[k]; c.top_right[k] = topRight[k]; c.bottom_left[k] = bottomLeft[k];
      c.right[k] = right[k]; c.up[k] = up[k]; c.ahead[k] = ahead[k];
    }
    return c;
  }
  prt_postfx PostFx(bool enabled) const {
    prt_postfx p{};
    p.enabled = enabled ? 1 : 0;
    p.aberration = abberationIntensity;
    p.fov = fov; p.distortion = distortion;
    p.vignette_intensity = vignetteIntensity; p.vignette_radius = vignetteRadius;
    for (int k = 0; k < 4; k++) p.color_grading[k] = colorGrading[k];
    return p;
  }
};

// Renderer (Core/Renderer.h:12-112): the public switches of the reference and Tick()
class Renderer {
 public:
  enum class RENDER_STATES { BRDF, BASECOLOR, GEOMETRYNORMAL, SHADINGNORMAL, METAL, ROUGHNESS, EMMISIVE };

  bool accumulates = true;
  int bounces = 2;
  RENDER_STATES renderingMode = RENDER_STATES::BRDF;
  bool LIGHTED = true, GAMMACORRECTED = true, NORMALMAPPED = true, SKYBOX = true, AA = true, isStochastic = true;
  bool isPostProcessed = false;

  Scene scene;
  Camera camera;
  std::vector<float> accumulator;  // float4 x W*H: accumulator / samplesPerPixel (the displayed average)
  std::vector<uint32_t> screen;    // 0x00RRGGBB x W*H (RGBF32_to_RGB8 of the average)

  Renderer(int32_t width, int32_t height, int32_t device = 0) : width_(width), height_(height) {
    prt_device_desc d{device, 0};
    check(prt_create(&d, &ctx_));
    accumulator.assign(4 * (size_t)width * height, 0.0f);
    screen.assign((size_t)width * height, 0u);
  }
  // One process, several GPUs (prt_create_group): pixel tiles of tile x tile rendered concurrently on the
  // devices (a device may repeat), gathered on devices[0]; accumulator / screen hold the whole frame.
  Renderer(int32_t width, int32_t height, const std::vector<int32_t>& devices, int32_t tile = 32)
      : width_(width), height_(height) {
    std::vector<prt_device_desc> d;
    for (int32_t dev : devices) d.push_back(prt_device_desc{dev, 0});
    check(prt_create_group(d.data(), (int32_t)d.size(), tile, &ctx_));
    accumulator.assign(4 * (size_t)width * height, 0.0f);
    screen.assign((size_t)width * height, 0u);
  }
  // One process per GPU: rank 0 calls UniqueId(), the host program carries the bytes to the other ranks
  // (MPI, a socket, a file), and every rank calls JoinRccl before Init().  Tick() then renders this rank's
  // tiles and gathers the frame on rank 0 (accumulator / screen are filled on rank 0 only).
  static std::vector<uint8_t> UniqueId() {
    std::vector<uint8_t> id(PRT_SHARD_ID_BYTES);
    check(prt_shard_unique_id(id.data()));
    return id;
  }
  void JoinRccl(const std::vector<uint8_t>& id, int32_t rank, int32_t world, int32_t tile = 32) {
    if (id.size() != PRT_SHARD_ID_BYTES) throw Error(PRT_ERR_INVALID_ARGUMENT, "RCCL id must be 128 bytes");
    check(prt_shard_init_rccl(ctx_, id.data(), rank, world, tile));
  }
  ~Renderer() { prt_destroy(ctx_); }
  Renderer(const Renderer&) = delete;
  Renderer& operator=(const Renderer&) = delete;

  // Renderer::Init (Core/Renderer.cpp:7-16): scene + camera to the device, fresh accumulation state
  void Init() {
    scene.Upload(ctx_);
    const prt_camera c = camera.Plane();
    check(prt_set_camera(ctx_, &c));
    check(prt_reset_accumulation(ctx_, 1));
    frame_ = 0;
  }

  // Renderer::Tick (Core/Renderer.cpp:22-148): `frames` reference frames (2 camera paths per pixel each
  // with AA) folded into the progressive accumulator; accumulator / screen hold the result afterwards
  void Tick(float deltaTime = 0.0f, int32_t frames = 1) {
    (void)deltaTime;
    prt_render_params p{};
    p.width = width_;
    p.height = height_;
    p.spp = frames * (AA ? 2 : 1);
    p.bounces = bounces;
    p.flags = Flags();
    p.render_mode = (int32_t)renderingMode;
    p.frame_index = frame_;
    p.seed = 0;
    const prt_postfx pf = camera.PostFx(isPostProcessed);
    check(prt_set_postfx(ctx_, &pf));
    check(prt_render(ctx_, &p, accumulator.data(), screen.data(), 0u, &stats_));
    if (stats_.stack_overflows)  // a dropped traversal stack group may have lost hits (prt_stats)
      throw Error(PRT_ERR_HIP, "traversal stack overflow: " + std::to_string(stats_.stack_overflows) +
                                        " node groups dropped");
    frame_ += (uint32_t)frames;
  }

  // Tick with the outputs in device memory (float4 average, 0x00RRGGBB) and no stats: no host wait.  With frames
  // in flight (SetFramesInFlight(n > 1), ABI 9) consecutive calls overlap on internal streams and a call's outputs
  // are complete in the context stream's order once n - 1 more calls are made, or after Finish(); the
  // accumulation stays in call order, so the images equal Tick()'s
  void TickDevice(float* avg_dev, uint32_t* rgb8_dev, int32_t frames = 1) {
    prt_render_params p{};
    p.width = width_;
    p.height = height_;
    p.spp = frames * (AA ? 2 : 1);
    p.bounces = bounces;
    p.flags = Flags();
    p.render_mode = (int32_t)renderingMode;
    p.frame_index = frame_;
    p.seed = 0;
    const prt_postfx pf = camera.PostFx(isPostProcessed);
    check(prt_set_postfx(ctx_, &pf));
    check(prt_render(ctx_, &p, avg_dev, rgb8_dev, PRT_OUT_DEVICE, nullptr));
    frame_ += (uint32_t)frames;
  }
  void SetFramesInFlight(int32_t n) { check(prt_set_frames_in_flight(ctx_, n)); }
  void Finish() { check(prt_finish(ctx_)); }  // the frames in flight joined into the context stream

  // Camera::HandleInput returned true: new screen plane, accumulator memset (Core/Renderer.cpp:147)
  void CameraMoved() {
    const prt_camera c = camera.Plane();
    check(prt_set_camera(ctx_, &c));
    check(prt_reset_accumulation(ctx_, 0));
  }

  // checkpoint of a long progressive render: the accumulation blob (prt_save_accumulation) and the frame counter
  // the RNG stream continues from; Resume(blob, frame) before the next Tick continues bit for bit
  std::vector<uint8_t> Checkpoint(uint32_t* frame) const {
    uint64_t n = 0;
    check(prt_accumulation_bytes(ctx_, &n));
    std::vector<uint8_t> blob(n);
    if (n) check(prt_save_accumulation(ctx_, blob.data(), n));
    if (frame) *frame = frame_;
    return blob;
  }
  void Resume(const std::vector<uint8_t>& blob, uint32_t frame) {
    check(prt_load_accumulation(ctx_, blob.data(), blob.size()));
    frame_ = frame;
  }

  // rays traced since construction (or the last reset): the reference's ImGui ray counter (Core/Renderer.cpp:467-474)
  void RayTotals(uint64_t* segments, uint64_t* shadow_rays, bool reset = false) const {
    check(prt_ray_totals(ctx_, segments, shadow_rays, reset ? 1 : 0));
  }

  uint32_t Flags() const {
    return (AA ? PRT_FLAG_AA : 0u) | (accumulates ? PRT_FLAG_ACCUMULATE : 0u) | (GAMMACORRECTED ? PRT_FLAG_GAMMA : 0u) |
           (NORMALMAPPED ? PRT_FLAG_NORMALMAP : 0u) | (SKYBOX ? PRT_FLAG_SKYBOX : 0u) | (LIGHTED ? PRT_FLAG_LIGHTED : 0u) |
           (isStochastic ? PRT_FLAG_STOCHASTIC : 0u);
  }
  const prt_stats& LastStats() const { return stats_; }
  prt_ctx* Context() const { return ctx_; }
  int32_t Width() const { return width_; }
  int32_t Height() const { return height_; }

 private:
  prt_ctx* ctx_ = nullptr;
  int32_t width_, height_;
  uint32_t frame_ = 0;
  prt_stats stats_{};
};

}  // namespace prt
