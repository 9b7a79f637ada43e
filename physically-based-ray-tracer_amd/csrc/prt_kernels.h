// prt_kernels.h -- the path-tracing kernels (Renderer::Tick pixel loop + Renderer::Trace).
#pragma once
#include "prt_shade.h"
#include "prt_traverse.h"

namespace prt {

constexpr int kBlock = 256;

// work-item -> pixel mapping.  The image is cut into ts x ts distribution tiles (row-major tile ids);
// rank r of 'world' owns tiles r, r+world, ...  Inside a tile, 64 consecutive items form an 8x8 pixel
// block (one wave = one 8x8 block: coherent primary rays).  world = 1, ts = 8 is the single-GPU case.
struct TileMap {
  int32_t W, H, ts, rank, world;
  int32_t tiles_x, tiles_y, local_tiles;
  uint32_t items;  // per frame = local_tiles * ts * ts
};

__host__ __device__ inline TileMap make_tilemap(int32_t W, int32_t H, int32_t ts, int32_t rank, int32_t world) {
  TileMap m;
  m.W = W; m.H = H; m.ts = ts; m.rank = rank; m.world = world;
  m.tiles_x = (W + ts - 1) / ts;
  m.tiles_y = (H + ts - 1) / ts;
  const int32_t n = m.tiles_x * m.tiles_y;
  m.local_tiles = rank < n ? (n - rank + world - 1) / world : 0;
  m.items = (uint32_t)m.local_tiles * (uint32_t)(ts * ts);
  return m;
}
// returns false when the item's pixel lies outside the image
__host__ __device__ inline bool item_pixel(const TileMap& m, uint32_t r, int32_t& px, int32_t& py) {
  const uint32_t tsq = (uint32_t)(m.ts * m.ts);
  const uint32_t lt = r / tsq, k = r % tsq;
  const uint32_t g = (uint32_t)m.rank + lt * (uint32_t)m.world;
  const uint32_t gx = g % (uint32_t)m.tiles_x, gy = g / (uint32_t)m.tiles_x;
  const uint32_t sub = k >> 6, lane = k & 63u, spr = (uint32_t)(m.ts >> 3);
  px = (int32_t)(gx * m.ts + (sub % spr) * 8 + (lane & 7u));
  py = (int32_t)(gy * m.ts + (sub / spr) * 8 + (lane >> 3));
  return px < m.W && py < m.H;
}

// pixels of the image inside rank's tiles (items minus the overhang of partial tiles at the right / bottom edge)
inline uint64_t tile_image_pixels(const TileMap& m) {
  uint64_t n = 0;
  for (int32_t lt = 0; lt < m.local_tiles; lt++) {
    const int32_t g = m.rank + lt * m.world, gx = g % m.tiles_x, gy = g / m.tiles_x;
    const int32_t w = m.W - gx * m.ts < m.ts ? m.W - gx * m.ts : m.ts;
    const int32_t h = m.H - gy * m.ts < m.ts ? m.H - gy * m.ts : m.ts;
    n += (uint64_t)w * (uint64_t)h;
  }
  return n;
}

struct TraceArgs {
  int32_t W, H;
  int32_t bounces;
  uint32_t flags;
  int32_t mode;
  uint32_t frame_index;
  uint32_t seed;
  int32_t frames;
};

}  // namespace prt
