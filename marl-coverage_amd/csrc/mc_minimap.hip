// mc_minimap.hip — the minimap obs layers of DecGridRL (mini_map_rad > 0,
// dec_grid_rl.py:360-370):
//   z[i][3] = cv2.resize(arraySubset(_free_pad[i], x, y, m), (E, E), INTER_LINEAR)
//   z[i][4] = cv2.resize(arraySubset(_obst_pad[i], x, y, m), (E, E), INTER_LINEAR)
// (they overwrite the dist / dijkstra layer at 3).  OpenCV's generic CV_64F
// path, as oracle/cpu_ref.py:cv2_resize_linear restates it: a horizontal pass
// S[r][xofs]*a0 + S[r][xofs+1]*a1 (a copy of S[r][xofs] from xmax on), then
// a vertical pass H[r0]*b0 + H[r1]*b1 with the rows clipped — double
// arithmetic, float weights (host-built taps, MinimapTaps), no FMA (explicit
// __dmul_rn / __dadd_rn: hipcc contracts a*b + c otherwise).  Parity with
// real OpenCV is unpinned.
//
// One thread per (env, agent, layer, output cell); the source cells are bits
// of the post-step tile maps (cells outside the padded grid are 0: the pad
// ring of _free_pad / _obst_pad is never marked).  Output float64
// [B][N][2][E][E] (mc_set_minimap_obs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_device.h"

namespace mc {

struct MinimapTaps {
  int n;     // source side 2m + 1
  int E;     // destination side
  int m;     // mini_map_rad
  int copy;  // n == E: cv::resize copies
  int xmax;
  int xofs[32];
  float a0[32], a1[32];
  int r0[32], r1[32];  // clipped source rows
  float b0[32], b1[32];
};

__device__ __forceinline__ double mm_src(const State& s, const uint64_t* map, int x, int y) {
  if (x < 0 || y < 0 || x >= s.Wp || y >= s.Lp) return 0.0;
  return (double)((map[tile_index(s.TCS, x >> 3, y >> 3)] >> tile_bit(x, y)) & 1ull);
}

__global__ __launch_bounds__(256) void minimap_kernel(State s, MinimapTaps T, double* __restrict__ out) {
  const int E = T.E, per_agent = 2 * E * E;
  const size_t total = (size_t)s.B * s.N * per_agent;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t ea = i / per_agent;
    const int rem = (int)(i - ea * per_agent);
    const int layer = rem / (E * E), cell = rem - layer * E * E;
    const int dy = cell / E, dx = cell - dy * E;
    const int2 p = reinterpret_cast<const int2*>(s.pos)[ea];
    const uint64_t* map = (layer == 0 ? s.freem : s.obstm) + ea * (size_t)s.MT;
    const int x0 = p.x - T.m, y0 = p.y - T.m;  // crop origin, padded-grid coordinates
    double v;
    if (T.copy) {
      v = mm_src(s, map, x0 + dy, y0 + dx);
    } else {
      const int sx = T.xofs[dx];
      double h[2];
      const int rr[2] = {T.r0[dy], T.r1[dy]};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const double s0 = mm_src(s, map, x0 + rr[k], y0 + sx);
        if (dx < T.xmax) {
          const double s1 = mm_src(s, map, x0 + rr[k], y0 + sx + 1);
          h[k] = __dadd_rn(__dmul_rn(s0, (double)T.a0[dx]), __dmul_rn(s1, (double)T.a1[dx]));
        } else {
          h[k] = s0;
        }
      }
      v = __dadd_rn(__dmul_rn(h[0], (double)T.b0[dy]), __dmul_rn(h[1], (double)T.b1[dy]));
    }
    out[i] = v;
  }
}

// OpenCV's INTER_LINEAR taps (resizeGeneric_ set-up, non-area mode), the
// float arithmetic of oracle/cpu_ref.py:_linear_taps
MinimapTaps minimap_taps(int m, int E) {
  MinimapTaps T{};
  T.n = 2 * m + 1;
  T.E = E;
  T.m = m;
  T.copy = T.n == E;
  const double inv_scale = (double)E / (double)T.n;
  const double scale = 1.0 / inv_scale;
  T.xmax = E;
  for (int d = 0; d < E; ++d) {
    float f = (float)((d + 0.5) * scale - 0.5);
    const int sy = (int)floorf(f);
    f -= (float)sy;
    T.b0[d] = 1.0f - f;
    T.b1[d] = f;
    T.r0[d] = sy < 0 ? 0 : (sy > T.n - 1 ? T.n - 1 : sy);
    T.r1[d] = sy + 1 < 0 ? 0 : (sy + 1 > T.n - 1 ? T.n - 1 : sy + 1);
    float fx = f;
    int sx = sy;
    if (sx < 0) {
      fx = 0.0f;
      sx = 0;
    }
    if (sx + 1 >= T.n) {
      if (d < T.xmax) T.xmax = d;
      if (sx >= T.n - 1) {
        fx = 0.0f;
        sx = T.n - 1;
      }
    }
    T.xofs[d] = sx;
    T.a0[d] = 1.0f - fx;
    T.a1[d] = fx;
  }
  return T;
}

hipError_t launch_minimap(const State& s, int mini, double* out, hipStream_t stream) {
  const MinimapTaps T = minimap_taps(mini, s.E);
  const size_t total = (size_t)s.B * s.N * 2 * s.E * s.E;
  size_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(minimap_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, s, T, out);
  return hipGetLastError();
}

}  // namespace mc
