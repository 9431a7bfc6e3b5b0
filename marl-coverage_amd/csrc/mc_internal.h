// mc_internal.h — device-side state descriptor shared by the kernels and the
// C ABI (mc_capi.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mc {

enum Mode : int { MODE_STEP = 0, MODE_RESET = 1 };

// Device error bits (OR-ed into State::err, read by mc_check).
enum : uint32_t {
  ERR_WINDOW = 1u << 0,     // a beam left its staged window (cannot happen:
                            // every lidar cell is within Chebyshev ceil(range))
  ERR_PLACEMENT = 1u << 2,  // could not place all robots on free cells
  ERR_INJECT = 1u << 3,     // injected start cell invalid (obstacle / clash)
};

// One lidar beam, derived on the host from the reference's (xinc, yinc,
// distinc) row (lidar.py:38-48).  One of |xinc|, |yinc| is exactly 1, so the
// march moves exactly +-1 per step along that "major" axis; the minor
// coordinate is the float64 chain  m_0 = start, m_{k+1} = m_k + minor  and the
// visited cell is int(m_k).  Because |minor| <= 1, int(m_{k+1}) - int(m_k) is
// 0 or sign(minor): the host runs the reference's exact float64 `+=` chain for
// every integer start coordinate and stores bit k of beam_bits[b][start] =
// "the minor cell moves at step k".  K = number of `currdist += distinc`
// steps before `currdist < range` fails (position independent): the beam
// visits cells k = 0..K unless an obstacle stops it.
struct Beam {
  int32_t K;
  int16_t axis;   // 0: major axis is x (rows), 1: major axis is y (columns)
  int16_t sign;   // +1 / -1 along the major axis
  int32_t msign;  // +1 / -1 / 0: direction of a minor-axis move
  int32_t pad_;
};
static_assert(sizeof(Beam) == 16, "Beam is 16 bytes");

// Everything a kernel needs, passed by value.  Layout (all device memory):
//   grid_neg/grid_pos  u64 [G][Wp][nw]     bit y%64 of word y/64 = cell (x,y)
//   freem/obstm        u64 [B][N][Wp][nw]  per-agent _free_pad/_obst_pad
//                                          (padded-grid region only: the
//                                          reference never marks the pad ring)
//   vis                u64 [B][Wp][nw]     _visited (union of free maps)
//   pos                i32 [B][N][2]       (_xinds, _yinds)
struct State {
  int B, N, Wp, Lp, nw, G;
  int H;                   // sensing half-width (>= egoradius)
  int We;                  // staged rows/cols per agent: 2H+3 (window +-1 for the move)
  uint32_t mg_We, mg_LcE, mg_E, mg_nb;  // magic reciprocals: n / d == umulhi(n, mg_d)
  int ego, E, Lc;          // egoradius, obs side, obs layers
  int sensor, nbeams, sq_r;
  double pen, term, dincr;
  int maxsteps, comm_r, sst, auto_reset, grid_mode;
  uint64_t seed;

  const uint64_t* grid_neg;
  const uint64_t* grid_pos;
  const int32_t* numfree;
  const Beam* beams;
  const uint64_t* beam_bits;  // [nbeams][bcmax] minor-move bits per start coordinate
  int bcmax;                  // max(Wp, Lp)
  int beam_kmax;              // max Beam::K (<= H): march steps of a pass
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
  uint64_t* stamps;        // diagnostic builds (-DMC_STAMPS) only: [B][16] s_memtime
};

constexpr int kMaxItemsPerLane = 2;  // staged (agent, row) items per lane

// floor(n / d) == umulhi(n, magic(d)) for 2 <= d < 2^16 and n * d < 2^32;
// d == 1 (2^32 does not fit) is encoded as 0 and handled by the caller
__host__ __device__ constexpr uint32_t magic_div(uint32_t d) {
  return d <= 1 ? 0u : (uint32_t)((0x100000000ull + d - 1) / d);
}

// Compile-time shape of an env kernel instantiation: fields > 0 are baked in
// (loop bounds, divisions and LDS offsets fold to constants and the march
// unrolls); 0 leaves the field to the runtime State.  The launcher picks a
// specialised instantiation only when the runtime State matches it exactly.
template <int N_, int H_, int NB_, int EGO_, int KM_>
struct Shape {
  static constexpr int N = N_, H = H_, NB = NB_, EGO = EGO_, KM = KM_;
  __host__ __device__ static bool matches(const struct State& s);
};

// LDS bytes of the env kernel (host + device use the same carve).
__host__ __device__ inline size_t env_lds_bytes(int N, int We, int nbeams, int Lc, int E,
                                                size_t wbytes) {
  const size_t items = (size_t)N * We;
  size_t b = (6 * items * wbytes + 15) & ~(size_t)15;  // neg, pos, fold, oold, fp, op
  b += (size_t)(nbeams > 0 ? nbeams : 1) * 16;  // beams
  b += (size_t)N * 16;                       // x0, y0, x, y
  b += 64;                                   // scalars
  b += ((size_t)N + 15) & ~(size_t)15;       // actions
  b += (((size_t)N * Lc * E) + 15) & ~(size_t)15;  // obs rows (one E-bit byte each)
  b = (b + 15) & ~(size_t)15;
  b += 64 * wbytes;  // per-lane sink word for masked-off lidar marks
  return b;
}

template <int N_, int H_, int NB_, int EGO_, int KM_>
__host__ __device__ inline bool Shape<N_, H_, NB_, EGO_, KM_>::matches(const State& s) {
  return (N_ == 0 || s.N == N_) && (H_ == 0 || s.H == H_) &&
         (NB_ == 0 || (s.sensor == 0 && s.nbeams == NB_)) && (EGO_ == 0 || s.ego == EGO_) &&
         (KM_ == 0 || (s.sensor == 0 && s.beam_kmax == KM_));
}

// overwrite the baked-in fields of a kernel's State copy with constants
template <class SH>
__device__ __forceinline__ void specialize(State& s) {
  if constexpr (SH::N > 0) s.N = SH::N;
  if constexpr (SH::H > 0) {
    s.H = SH::H;
    s.We = 2 * SH::H + 3;
    s.mg_We = magic_div(2 * SH::H + 3);
  }
  if constexpr (SH::NB > 0) {
    s.sensor = 0;
    s.nbeams = SH::NB;
    s.mg_nb = magic_div(SH::NB);
  }
  if constexpr (SH::EGO > 0) {
    s.ego = SH::EGO;
    s.E = 2 * SH::EGO + 1;
    s.Lc = 3;
    s.mg_E = magic_div(2 * SH::EGO + 1);
    s.mg_LcE = magic_div(3 * (2 * SH::EGO + 1));
  }
  if constexpr (SH::KM > 0) s.beam_kmax = SH::KM;
}

}  // namespace mc
