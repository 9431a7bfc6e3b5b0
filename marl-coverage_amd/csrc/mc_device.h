// mc_device.h — small device helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_internal.h"

namespace mc {

// bits [off, off+64) of the 128-bit value hi:lo
__device__ __forceinline__ uint64_t funnel(uint64_t lo, uint64_t hi, int off) {
  return off ? ((lo >> off) | (hi << (64 - off))) : lo;
}

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

// isInBounds + grid < 0 (dec_grid_rl.py:284-295, :310) read from HBM
__device__ __forceinline__ bool grid_blocked(const State& s, int g, int x, int y) {
  if (x < 0 || y < 0 || x >= s.Wp || y >= s.Lp) return true;
  const uint64_t wv = s.grid_neg[((size_t)g * s.Wp + x) * s.nw + (y >> 6)];
  return (wv >> (y & 63)) & 1ull;
}

}  // namespace mc
