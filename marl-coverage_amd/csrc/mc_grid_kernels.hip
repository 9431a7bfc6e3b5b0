// mc_grid_kernels.hip — grid-pool upload/generation and map sharing.
//
//   pack_grids_kernel: int8 padded grids -> neg/pos bit planes + numfree
//                      (the np.pad / count_nonzero of dec_grid_rl.py:471,517)
//   gen_grids_kernel:  Bernoulli obstacle pool (Utils/gridmaker.py:127-128)
//   share_kernel:      DecGridRL.shareMaps (dec_grid_rl.py:423-447)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_device.h"

namespace mc {

// --------------------------------------------------------------------------
// shareMaps (dec_grid_rl.py:423-447), run before the step kernel when
// map_sharing is on: agent i's maps <- OR over {j: adj(i,j) or i==j}, with
// adj from the positions at the start of the step (the last comm graph).
// grid = (ceil(TR*TC / 64), B); block = 64 lanes, one tile position each.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(64) void share_kernel(State s, const uint8_t* __restrict__ actions) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int e = blockIdx.y;
  const int N = s.N;
  if (actions[(size_t)e * N] == 255) return;  // sentinel: no state change
  const size_t mw = (size_t)s.MT;
  const int lane = threadIdx.x;
  const size_t w = (size_t)blockIdx.x * 64 + lane;
  uint64_t* fo = reinterpret_cast<uint64_t*>(smem);   // [N][64]
  uint64_t* oo = fo + (size_t)N * 64;                  // [N][64]
  int32_t* px = reinterpret_cast<int32_t*>(oo + (size_t)N * 64);
  int32_t* py = px + 64;
  if (lane < N) {
    px[lane] = s.pos[((size_t)e * N + lane) * 2];
    py[lane] = s.pos[((size_t)e * N + lane) * 2 + 1];
  }
  uint64_t* f = s.freem + (size_t)e * N * mw + w;
  uint64_t* o = s.obstm + (size_t)e * N * mw + w;
  const bool live = w < mw;
  for (int j = 0; j < N; ++j) {
    fo[j * 64 + lane] = live ? f[j * mw] : 0ull;
    oo[j * 64 + lane] = live ? o[j * mw] : 0ull;
  }
  __syncthreads();
  if (!live) return;
  uint32_t cnt = 0;
  for (int i = 0; i < N; ++i) {
    uint64_t fn = 0, on = 0;
    for (int j = 0; j < N; ++j) {
      const int d = max(abs(px[i] - px[j]), abs(py[i] - py[j]));
      if (d <= s.comm_r || i == j) {
        fn |= fo[j * 64 + lane];
        on |= oo[j * 64 + lane];
      }
    }
    const uint64_t fi = fo[i * 64 + lane], oi = oo[i * 64 + lane];
    cnt += __popcll(fn & ~fi);
    if (fn != fi) f[i * mw] = fn;
    if (on != oi) o[i * mw] = on;
  }
  if (cnt) atomicAdd(&s.free_cnt[e], cnt);
}

// --------------------------------------------------------------------------
// grid pool upload / generation
// --------------------------------------------------------------------------
// int8 [G][Wp][Lp] -> neg/pos tiles, numfree[g] = count(grid > 0).  Cells of
// an edge tile beyond the grid are obstacles (isInBounds).
__global__ void pack_grids_kernel(State s, const int8_t* __restrict__ grids) {
  const size_t mt = (size_t)s.MT;
  const size_t total = (size_t)s.G * mt;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int g = (int)(i / mt);
    const size_t rem = i - (size_t)g * mt;
    // tile_index inverse: 4x4-tile blocks, row-major
    const int blk = (int)(rem >> 4), in = (int)(rem & 15);
    const int ti = (blk / s.TCS) * 4 + (in >> 2), tj = (blk % s.TCS) * 4 + (in & 3);
    uint64_t neg = 0, pos = 0;
    for (int r = 0; r < 8; ++r) {
      const int x = 8 * ti + r;
      for (int c = 0; c < 8; ++c) {
        const int y = 8 * tj + c;
        const uint64_t bit = 1ull << (8 * r + c);
        if (x >= s.Wp || y >= s.Lp) { neg |= bit; continue; }
        const int8_t v = grids[((size_t)g * s.Wp + x) * s.Lp + y];
        if (v < 0) neg |= bit;
        if (v > 0) pos |= bit;
      }
    }
    const_cast<uint64_t*>(s.grid_neg)[i] = neg;
    const_cast<uint64_t*>(s.grid_pos)[i] = pos;
    if (pos) atomicAdd(const_cast<int32_t*>(&s.numfree[g]), (int32_t)__popcll(pos));
  }
}

// Bernoulli(p) obstacles in the interior, -1 border (gridgen semantics,
// Utils/gridmaker.py:127-128, plus the np.pad of dec_grid_rl.py:471).  One
// Philox block per tile row: 8 cells x 32 bits = 2 calls.
__global__ void gen_grids_kernel(State s, uint64_t seed, uint32_t thresh, int all_free) {
  const size_t mt = (size_t)s.MT;
  const size_t total = (size_t)s.G * mt;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int g = (int)(i / mt);
    const size_t rem = i - (size_t)g * mt;
    // tile_index inverse: 4x4-tile blocks, row-major
    const int blk = (int)(rem >> 4), in = (int)(rem & 15);
    const int ti = (blk / s.TCS) * 4 + (in >> 2), tj = (blk % s.TCS) * 4 + (in & 3);
    uint64_t neg = 0;
    for (int r = 0; r < 8; ++r) {
      const int x = 8 * ti + r;
      for (int h = 0; h < 2; ++h) {
        const uint4 q = philox(seed, make_uint4(s.grid0 + (uint32_t)g, (uint32_t)x, (uint32_t)(tj * 2 + h), 0x67656e21u));
        const uint32_t rv[4] = {q.x, q.y, q.z, q.w};
        for (int t = 0; t < 4; ++t) {
          const int c = h * 4 + t;
          const int y = 8 * tj + c;
          const bool outside = x >= s.Wp || y >= s.Lp;
          const bool border = x == 0 || x == s.Wp - 1 || y == 0 || y == s.Lp - 1;
          if (outside || border || (!all_free && rv[t] < thresh)) neg |= 1ull << (8 * r + c);
        }
      }
    }
    const uint64_t pos = ~neg;  // outside cells are in neg
    const_cast<uint64_t*>(s.grid_neg)[i] = neg;
    const_cast<uint64_t*>(s.grid_pos)[i] = pos;
    if (pos) atomicAdd(const_cast<int32_t*>(&s.numfree[g]), (int32_t)__popcll(pos));
  }
}

// Synthetic actions (SURVEY 8(d) "Actions (GPU)"): agent i of env e at step
// t is bits 2i, 2i+1 of Philox(seed, (global env id, t)) -- one 128-bit draw
// per env covers N <= 64 agents.
__global__ void random_actions_kernel(State s, uint64_t seed, uint32_t step, uint8_t* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= s.B) return;
  const uint4 r = philox(seed, make_uint4(s.env0 + (uint32_t)e, step, 0u, 0x61637473u));
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint8_t* o = out + (size_t)e * s.N;
  for (int i = 0; i < s.N; ++i) o[i] = (uint8_t)((w[i >> 4] >> (2 * (i & 15))) & 3u);
}

hipError_t launch_random_actions(const State& s, uint64_t seed, int step, uint8_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(random_actions_kernel, dim3((s.B + 255) / 256), dim3(256), 0, stream, s, seed,
                     (uint32_t)step, out);
  return hipGetLastError();
}

hipError_t launch_share(const State& s, const uint8_t* actions, hipStream_t stream) {
  const size_t mw = (size_t)s.MT;
  dim3 grid((unsigned)((mw + 63) / 64), s.B), block(64);
  const size_t lds = (size_t)s.N * 64 * 16 + 64 * 8;
  hipLaunchKernelGGL(share_kernel, grid, block, lds, stream, s, actions);
  return hipGetLastError();
}

hipError_t launch_pack(const State& s, const int8_t* grids, hipStream_t stream) {
  const size_t total = (size_t)s.G * s.MT;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(pack_grids_kernel, dim3(blocks), dim3(256), 0, stream, s, grids);
  return hipGetLastError();
}

hipError_t launch_gen(const State& s, uint64_t seed, double p, hipStream_t stream) {
  const size_t total = (size_t)s.G * s.MT;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  double t = p * 4294967296.0;
  uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (t <= 0.0 ? 0u : (uint32_t)t);
  hipLaunchKernelGGL(gen_grids_kernel, dim3(blocks), dim3(256), 0, stream, s, seed, thresh,
                     p <= 0.0 ? 1 : 0);
  return hipGetLastError();
}

}  // namespace mc
