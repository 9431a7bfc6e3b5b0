// mc_device.h — small device helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_internal.h"

namespace mc {

__device__ __forceinline__ uint64_t low_mask(int w) {
  return w >= 64 ? ~0ull : ((1ull << w) - 1ull);
}

// Philox4x32-10 (Salmon et al., SC'11).
__device__ __forceinline__ uint4 philox(uint64_t seed, uint4 c) {
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// floor(r * n / 2^32): a uniform draw in [0, n) from 32 random bits
__device__ __forceinline__ uint32_t bounded(uint32_t r, uint32_t n) {
  return (uint32_t)(((uint64_t)r * n) >> 32);
}

// distance_map value (dec_grid_rl.py:260-282) of a cell at L1 distance d
// when the map maximum is M, in the reference's float32 steps
__device__ __forceinline__ float dist_value(float d, float M) {
  return M > 0.0f ? __fsub_rn(1.0f, __fdiv_rn(d, M)) : __fsub_rn(1.0f, d);
}

// dist_reward witness cell of a packed (x << 16) | (y & 0xFFFF) word (map
// coordinates, signed 16-bit halves: the witness may lie in the pad ring)
__device__ __forceinline__ int witness_x(int32_t w) { return w >> 16; }
__device__ __forceinline__ int witness_y(int32_t w) { return (int)(int16_t)(w & 0xFFFF); }
__device__ __forceinline__ int32_t pack_witness(int x, int y) {
  return (int32_t)(((uint32_t)x << 16) | ((uint32_t)y & 0xFFFFu));
}

// true when a set bit of tile nb (cell (r, c) = map cell (x0 + r, y0 + c))
// lies at L1 distance < M from map cell (wx, wy).  The tile's bounding box
// rejects almost every tile; the exact row-by-row test runs only near the
// witness.
__device__ __forceinline__ bool bits_within(uint64_t nb, int x0, int y0, int wx, int wy, int M) {
  const int bx = max(0, max(x0 - wx, wx - (x0 + 7)));
  const int by = max(0, max(y0 - wy, wy - (y0 + 7)));
  if (bx + by >= M || !nb) return false;
  // the set bits' bounding box (rows: a bit per nonzero byte; columns: the
  // OR of the bytes): no bit within M if the box is not, every bit within M
  // if its far corner is -- the row walk below only for the boxes between
  uint64_t t = nb | (nb >> 4);
  t |= t >> 2;
  t |= t >> 1;
  const uint32_t rows = (uint32_t)(((t & 0x0101010101010101ull) * 0x0102040810204080ull) >> 56);
  uint64_t c = nb | (nb >> 32);
  c |= c >> 16;
  c |= c >> 8;
  const uint32_t cols = (uint32_t)c & 0xFFu;
  const int r0 = x0 + __ffs(rows) - 1, r1 = x0 + 31 - __clz(rows);
  const int c0 = y0 + __ffs(cols) - 1, c1 = y0 + 31 - __clz(cols);
  const int lb = max(0, max(r0 - wx, wx - r1)) + max(0, max(c0 - wy, wy - c1));
  if (lb >= M) return false;
  if (max(abs(wx - r0), abs(wx - r1)) + max(abs(wy - c0), abs(wy - c1)) < M) return true;
  const int p = wy - y0;  // witness column relative to the tile
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)(nb >> (8 * r)) & 0xFFu;
    if (!row) continue;
    int dy;
    if (p < 0) dy = __ffs(row) - 1 - p;
    else if (p > 7) dy = p - (31 - __clz(row));
    else {
      const uint32_t lo = row & ((2u << p) - 1u), hi = row >> p;
      dy = lo ? p - (31 - __clz(lo)) : 8;
      if (hi) dy = min(dy, __ffs(hi) - 1);
    }
    if (abs(x0 + r - wx) + dy < M) return true;
  }
  return false;
}

// bit of cell (r, c) inside its 8x8 tile
__device__ __forceinline__ int tile_bit(int r, int c) { return ((r & 7) << 3) | (c & 7); }

// isInBounds + grid < 0 (dec_grid_rl.py:284-295, :310) read from HBM
__device__ __forceinline__ bool grid_blocked(const State& s, int g, int x, int y) {
  if (x < 0 || y < 0 || x >= s.Wp || y >= s.Lp) return true;
  const uint64_t t = s.grid_neg[(size_t)g * s.MT + tile_index(s.TCS, x >> 3, y >> 3)];
  return (t >> tile_bit(x, y)) & 1ull;
}

// cells of global tile (ti, tj) that lie inside the padded grid
__device__ __forceinline__ uint64_t tile_in_grid(const State& s, int ti, int tj) {
  const int rv = s.Wp - 8 * ti, cv = s.Lp - 8 * tj;
  if (rv >= 8 && cv >= 8) return ~0ull;
  if (rv <= 0 || cv <= 0) return 0ull;
  const uint64_t cols = (cv >= 8 ? 0xFFull : ((1ull << cv) - 1ull)) * 0x0101010101010101ull;
  return cols & low_mask(8 * (rv >= 8 ? 8 : rv));
}

// rows [r0, r1] x cols [c0, c1] of a tile (inclusive, clamped to 0..7; empty
// when r1 < r0 or c1 < c0)
__device__ __forceinline__ uint64_t tile_rect(int r0, int r1, int c0, int c1) {
  r0 = r0 < 0 ? 0 : r0;
  c0 = c0 < 0 ? 0 : c0;
  r1 = r1 > 7 ? 7 : r1;
  c1 = c1 > 7 ? 7 : c1;
  if (r1 < r0 || c1 < c0) return 0ull;
  const uint64_t cols = (low_mask(c1 + 1) & ~low_mask(c0)) * 0x0101010101010101ull;
  return cols & low_mask(8 * (r1 + 1)) & ~low_mask(8 * r0);
}

}  // namespace mc
