// mc_bitboard.h — whole-map row bitboards for the kernels that need a map
// wider than the staged window (the dijkstra_input and dist_reward layers).
//
// The reference builds those layers on free_pad / obst_pad, which are the
// padded grid plus a `pad` ring on every side (dec_grid_rl.py:506-511).  Here
// that "extended grid" is RX = Wp + 2*pad rows of RY = Lp + 2*pad cells, one
// bit per cell, 64 columns per u64 word: extended cell (u, v) = map cell
// (u - pad, v - pad); the pad ring holds no marks.
#pragma once
#include "mc_device.h"

namespace mc {

// bits [64w, 64w + 64) of extended row u of a tiled map (tile_index order)
__device__ __forceinline__ uint64_t row_word(const State& s, const uint64_t* tiles, int pad, int u,
                                             int w) {
  uint64_t out = 0;
  const int X = u - pad;
  if (X < 0 || X >= s.Wp) return 0;
  const int Y0 = 64 * w - pad;  // map column of bit 0
  const int tj0 = Y0 < 0 ? 0 : (Y0 >> 3), tj1 = min((Y0 + 63) >> 3, s.TC - 1);
  const int sh = (X & 7) * 8;
  for (int tj = tj0; tj <= tj1; ++tj) {
    const uint64_t b = (tiles[tile_index(s.TCS, X >> 3, tj)] >> sh) & 0xFFull;
    const int off = 8 * tj - Y0;  // bit position of the tile's column 0
    out |= off >= 0 ? (b << off) : (b >> -off);
  }
  return out;
}

// 4-neighbourhood dilation of word i (row u, word w) of bitboard b
__device__ __forceinline__ uint64_t dilate_word(const uint64_t* b, int i, int u, int w, int RX,
                                                int RW) {
  const uint64_t c = b[i];
  uint64_t d = c | (c << 1) | (c >> 1);
  if (w > 0) d |= b[i - 1] >> 63;
  if (w < RW - 1) d |= b[i + 1] << 63;
  if (u > 0) d |= b[i - RW];
  if (u < RX - 1) d |= b[i + RW];
  return d;
}

}  // namespace mc
