// tile_map.h — index math shared by the kernels and the host layer: interleaved 32x32 tile
// sharding and division by launch-invariant divisors.
// Tiles of a W x H image are numbered row-major (GLRenderer::renderWavefront's tile order,
// /root/reference/src/GLRenderer.cpp:335-340); shard R of G owns tiles t with t % G == R.  A shard's
// pixels are tile-packed: local index l = (local tile) * 1024 + row-in-tile * 32 + column-in-tile.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SPTR_TM __host__ __device__ __forceinline__
#else
#define SPTR_TM inline
#endif

namespace sptr {

constexpr int kTileSize = 32;

SPTR_TM int tiles_x(int W) { return (W + kTileSize - 1) / kTileSize; }
SPTR_TM int tiles_total(int W, int H) { return tiles_x(W) * ((H + kTileSize - 1) / kTileSize); }
// number of tiles shard R of G owns
SPTR_TM uint32_t shard_tiles(int W, int H, int G, int R) { return (uint32_t)((tiles_total(W, H) - R + G - 1) / G); }
// tile-packed local index -> image pixel; false for slots of edge tiles outside the image
SPTR_TM bool shard_pixel(int W, int H, int G, int R, uint32_t l, int& x, int& y) {
  const uint32_t lt = l >> 10, w = l & 1023u;
  const uint32_t t = lt * (uint32_t)G + (uint32_t)R;
  const int ntx = tiles_x(W);
  x = (int)(t % (uint32_t)ntx) * kTileSize + (int)(w & 31u);
  y = (int)(t / (uint32_t)ntx) * kTileSize + (int)(w >> 5);
  return x < W && y < H;
}
// image pixel -> (owning shard, its local index)
SPTR_TM void pixel_shard(int W, int G, int x, int y, uint32_t& rank, uint32_t& l) {
  const uint32_t t = (uint32_t)(y / kTileSize) * (uint32_t)tiles_x(W) + (uint32_t)(x / kTileSize);
  rank = t % (uint32_t)G;
  l = (t / (uint32_t)G) * 1024u + (uint32_t)(y % kTileSize) * kTileSize + (uint32_t)(x % kTileSize);
}

// Division by a launch-invariant divisor d (1 <= d < 2^31) for numerators n < 2^30:
// q = (n * m) >> sh with sh = 31 + floor(log2 d), m = ceil(2^sh / d) <= 2^31.  Exact because
// n * (m*d - 2^sh) < 2^30 * 2^(s+1) = 2^sh  (tests/test_host_layer.py::test_fastdiv_exact).
struct FastDiv {
  uint32_t d, m, sh;
};
inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((2u << s) <= d && s < 31) ++s;  // s = floor(log2 d)
  const uint32_t sh = 31u + s;
  const unsigned __int128 one = 1;
  const uint64_t m = (uint64_t)(((one << sh) + d - 1) / d);
  return FastDiv{d, (uint32_t)m, sh};
}
SPTR_TM uint32_t fast_div(const FastDiv& f, uint32_t n) {
  return (uint32_t)(((uint64_t)n * (uint64_t)f.m) >> f.sh);
}

}  // namespace sptr
