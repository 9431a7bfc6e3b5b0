// mc_internal.h — device-side state descriptor shared by the kernels
// (mc_kernels.hip) and the C ABI (mc_capi.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

enum Mode : int { MODE_STEP = 0, MODE_RESET = 1 };

// Device error bits (OR-ed into State::err, read by mc_check).
enum : uint32_t {
  ERR_WINDOW = 1u << 0,     // a beam left its staged window (H too small)
  ERR_OUT_OF_GRID = 1u << 1,// a beam left the padded grid (unreachable with
                            // the -1 border: lidar.py:60-63 else-branch)
  ERR_PLACEMENT = 1u << 2,  // could not place all robots on free cells
  ERR_INJECT = 1u << 3,     // injected start cell invalid (obstacle / clash)
};

// Everything a kernel needs, passed by value.  Layout (all device memory):
//   grid_neg/grid_pos  u64 [G][Wp][nw]     bit y%64 of word y/64 = cell (x,y)
//   freem/obstm        u64 [B][N][Wp][nw]  per-agent _free_pad/_obst_pad
//                                          (only the padded-grid region: the
//                                          reference never marks the pad ring)
//   vis                u64 [B][Wp][nw]     _visited (union of free maps)
//   pos                i32 [B][N][2]       (_xinds, _yinds)
struct State {
  int B, N, Wp, Lp, nw, G;
  int H, Wwin;             // staged window half-width, rows per agent (2H+1)
  int ego, E, Lc;          // egoradius, obs side, obs layers
  int sensor, nbeams, sq_r;
  double range;
  double pen, term, dincr;
  int maxsteps, comm_r, sst, auto_reset, grid_mode;
  uint64_t seed;

  const uint64_t* grid_neg;
  const uint64_t* grid_pos;
  const int32_t* numfree;
  const double* beams;     // [nbeams][3] (xinc, yinc, distinc)
  int32_t* env_grid;
  int32_t* pos;
  uint64_t* moved;
  uint64_t* freem;
  uint64_t* obstm;
  uint64_t* vis;
  uint32_t* free_cnt;
  uint32_t* vis_cnt;
  int32_t* currstep;
  double* done_thresh;
  uint32_t* episode;
  uint32_t* err;
};

// LDS bytes the env kernel needs for this geometry (host + device).
__host__ __device__ inline size_t env_kernel_lds_bytes(int N, int Wwin) {
  size_t nw = (size_t)N * Wwin;
  // win_neg, win_pos, fpart, opart, fwin, owin : 6 x nw u64
  // rawf, rawo, rawu                            : 3 x 2nw u64
  // pos x/y (i32 x 2N), scalars block (64 B)
  size_t b = 6 * nw * 8 + 6 * nw * 8 + (size_t)N * 8 + 64;
  return (b + 15) & ~(size_t)15;
}

}  // namespace mc
