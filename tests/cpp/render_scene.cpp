// render_scene.cpp -- drives the C++ host mirror (include/prt_renderer.hpp) the way the reference's main
// loop drives Renderer: fill Scene + Camera, Init(), Tick() per frame.  Test program only: reads a scene
// written by tests/helpers.py::dump_scene and writes the accumulated float average + RGB8 frame.
//   usage: render_scene <scene.bin> <out.bin> <ticks> <bounces> [flags]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "prt_renderer.hpp"

namespace {

struct Reader {
  FILE* f;
  template <class T>
  T get() {
    T v;
    if (std::fread(&v, sizeof(T), 1, f) != 1) throw std::runtime_error("truncated scene file");
    return v;
  }
  template <class T>
  void arr(std::vector<T>& v, size_t n) {
    v.resize(n);
    if (n && std::fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("truncated scene file");
  }
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: render_scene <scene.bin> <out.bin> <ticks> <bounces> [flags] [shards]\n");
    return 2;
  }
  try {
    FILE* fp = std::fopen(argv[1], "rb");
    if (!fp) throw std::runtime_error("cannot open scene file");
    Reader r{fp};
    char magic[4];
    if (std::fread(magic, 1, 4, fp) != 4 || std::memcmp(magic, "PRTS", 4) != 0) throw std::runtime_error("bad magic");
    const int32_t W = r.get<int32_t>(), H = r.get<int32_t>();
    float pos[3], tgt[3];
    for (float& v : pos) v = r.get<float>();
    for (float& v : tgt) v = r.get<float>();
    const float aspect = r.get<float>();

    // shards > 1: one local group of that many tile shards on device 0 (prt_create_group)
    const int shards = argc > 6 ? std::atoi(argv[6]) : 1;
    std::unique_ptr<prt::Renderer> owner = shards > 1 ? std::make_unique<prt::Renderer>(W, H, std::vector<int32_t>(shards, 0), 16)
                                                       : std::make_unique<prt::Renderer>(W, H, 0);
    prt::Renderer& R = *owner;
    prt::Scene& S = R.scene;
    float* lw = &S.lights.point_pos[0][0];  // prt_lights is 39 consecutive floats
    for (int k = 0; k < 39; k++) lw[k] = r.get<float>();
    S.skyWidth = r.get<int32_t>();
    S.skyHeight = r.get<int32_t>();
    r.arr(S.skyPixels, 3 * (size_t)S.skyWidth * S.skyHeight);
    const int32_t ntex = r.get<int32_t>();
    S.textures.resize(ntex);
    for (prt::Texture& t : S.textures) {
      t.width = r.get<int32_t>();
      t.height = r.get<int32_t>();
      r.arr(t.pixels, (size_t)t.width * t.height);
    }
    const int32_t nm = r.get<int32_t>();
    S.models.resize(nm);
    for (prt::Model& m : S.models) {
      const int32_t T = r.get<int32_t>(), V = r.get<int32_t>();
      m.albedoTexture = r.get<int32_t>();
      m.normalTexture = r.get<int32_t>();
      m.metalnessTexture = r.get<int32_t>();
      m.emissionTexture = r.get<int32_t>();
      r.arr(m.triangles, 12 * (size_t)T);
      r.arr(m.fixedNormals, 12 * (size_t)T);
      r.arr(m.fixedTextureCoords, 6 * (size_t)T);
      r.arr(m.indices, 3 * (size_t)T);
      r.arr(m.vertices, 3 * (size_t)V);
      r.arr(m.faceNormals, 3 * (size_t)T);
    }
    const int32_t ni = r.get<int32_t>();
    S.gameobjects.resize(ni);
    for (prt::GameObject& g : S.gameobjects) {
      for (float& v : g.transform) v = r.get<float>();
      g.modelIndex = r.get<uint32_t>();
    }
    for (prt::GameObject& g : S.gameobjects) g.material = r.get<int32_t>();
    if (r.get<int32_t>()) {
      prt_area_light a{};
      float* aw = a.corner;  // corner, edge_u, edge_v, radiance: 12 consecutive floats
      for (int k = 0; k < 12; k++) aw[k] = r.get<float>();
      a.two_sided = r.get<int32_t>();
      S.areaLights.push_back(a);
    }
    std::fclose(fp);

    R.camera = prt::Camera(pos, tgt, aspect);
    R.bounces = std::atoi(argv[4]);
    if (argc > 5) {
      const unsigned fl = (unsigned)std::strtoul(argv[5], nullptr, 0);
      R.AA = fl & PRT_FLAG_AA; R.accumulates = fl & PRT_FLAG_ACCUMULATE; R.GAMMACORRECTED = fl & PRT_FLAG_GAMMA;
      R.NORMALMAPPED = fl & PRT_FLAG_NORMALMAP; R.SKYBOX = fl & PRT_FLAG_SKYBOX; R.LIGHTED = fl & PRT_FLAG_LIGHTED;
      R.isStochastic = fl & PRT_FLAG_STOCHASTIC;
    }
    R.Init();
    const int ticks = std::atoi(argv[3]);
    for (int t = 0; t < ticks; t++) R.Tick();
    FILE* fo = std::fopen(argv[2], "wb");
    if (!fo) throw std::runtime_error("cannot open output");
    std::fwrite(R.accumulator.data(), sizeof(float), R.accumulator.size(), fo);
    std::fwrite(R.screen.data(), sizeof(uint32_t), R.screen.size(), fo);
    std::fclose(fo);
    std::printf("render_scene: %dx%d ticks=%d segments=%llu shadow=%llu\n", W, H, ticks,
                (unsigned long long)R.LastStats().segments, (unsigned long long)R.LastStats().shadow_rays);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "render_scene: %s\n", e.what());
    return 1;
  }
  return 0;
}
