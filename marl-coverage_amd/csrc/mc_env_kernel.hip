// mc_env_kernel.hip — the step / reset kernel of the batched coverage env.
//
// Hot path restated from ExistentialRobotics/MARL-Coverage
//   Environments/dec_grid_rl.py  DecGridRL.step :91-169, reset :449-531
//   Environments/Sensors/lidar.py LidarSensor.getMeasurement :16-65
//   Environments/Sensors/squaresensor.py SquareSensor.getMeasurement :15-37
//
// A workgroup runs EPW envs ("slots"), LPE = NT / EPW lanes each.  Small envs
// (the BASELINE configs) pack two envs into one wave: every wave-wide
// instruction then serves two envs, which matters because the step is VALU
// issue bound.  Per env and step:
//   round trip 1  positions, actions, per-env scalars
//   round trip 2  for every agent the (2H+3)-row "extended window" around its
//                 pre-move cell: grid neg/pos bits, its free/obst mask words,
//                 the union (visited) words — 2 u64 per row and plane.  The
//                 +1 margin covers every post-move window, so the sequential
//                 moves, the beam march and the merge need no further loads.
//   LDS compute   moves (slot-serial in robot order), lidar or square sensing
//                 as LDS bit tests + ds_or marks, merge with popcounts
//   stores        changed mask words (plain stores: one writer per word),
//                 newly covered union bits (global_atomic_or: agents' windows
//                 overlap), positions, counters, reward, done, obs
// All float64 arithmetic is the reference's: rewards are assembled in
// reference order; the beam's float64 `+=` chain is encoded bit-exactly in
// the host-built step bits (mc_internal.h, struct Beam).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_device.h"
#include <cstdlib>

namespace mc {

#ifdef MC_STAMPS
#define STAMP(k)                                                                          \
  do {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                    \
    uint64_t _t;                                                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");            \
    if (threadIdx.x == 0 && s.stamps) s.stamps[(size_t)blockIdx.x * EPW * 16 + (k)] = _t; \
    __builtin_amdgcn_sched_barrier(0);                                                    \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#endif

// n / d via the magic reciprocal of mc_internal.h (magic == 0 encodes d == 1)
__device__ __forceinline__ int udiv(int n, uint32_t magic) {
  return magic ? (int)__umulhi((uint32_t)n, magic) : n;
}

__device__ __forceinline__ int rdlane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// Window rows are WT = uint32_t when 2H+3 <= 32 (every BASELINE config with
// range <= 14) and uint64_t otherwise.
template <typename WT>
__device__ __forceinline__ WT wmask_of(int w) { return (WT)low_mask(w); }
__device__ __forceinline__ int popc(uint32_t v) { return __popc(v); }
__device__ __forceinline__ int popc(uint64_t v) { return __popcll(v); }
__device__ __forceinline__ void lds_or(uint32_t* p, uint32_t v) { atomicOr((unsigned int*)p, v); }
__device__ __forceinline__ void lds_or(uint64_t* p, uint64_t v) { atomicOr((unsigned long long*)p, v); }

struct Scal {
  double pen;          // move penalties, accumulated in robot order
  double done_thresh;
  uint64_t moved;      // robots present in the reference's _robot_pad
  uint32_t cnt_free;   // newly set bits over all agents' free maps
  uint32_t cnt_vis;    // newly covered union cells (the obs reward)
  uint32_t free_old, vis_old;
  int32_t grid, numfree, currstep;
  uint32_t ep;
  int32_t do_reset;
  int32_t pad_;
};
static_assert(sizeof(Scal) <= 64, "Scal must fit its 64-byte LDS slot");

template <typename WT>
struct Lds {
  WT *neg, *pos, *fold, *oold, *fp, *op;
  Beam* beams;
  int32_t *x0, *y0, *x, *y;
  Scal* sc;
  uint8_t* act;
  uint8_t* obsrow;  // [N*Lc*E] E-bit crop rows
  WT* sink;         // [64] target of lidar marks a lane does not make
};

template <typename WT>
__device__ __forceinline__ Lds<WT> carve(char* smem, const State& s) {
  Lds<WT> L;
  const int items = s.N * s.We;
  WT* p = reinterpret_cast<WT*>(smem);
  L.neg = p;
  L.pos = p + items;
  L.fold = p + 2 * items;
  L.oold = p + 3 * items;
  L.fp = p + 4 * items;
  L.op = p + 5 * items;
  char* q = smem + ((6 * items * sizeof(WT) + 15) & ~(size_t)15);
  L.beams = reinterpret_cast<Beam*>(q);
  q += (size_t)(s.nbeams > 0 ? s.nbeams : 1) * 16;
  L.x0 = reinterpret_cast<int32_t*>(q);
  L.y0 = L.x0 + s.N;
  L.x = L.y0 + s.N;
  L.y = L.x + s.N;
  q += (size_t)s.N * 16;
  L.sc = reinterpret_cast<Scal*>(q);
  q += 64;
  L.act = reinterpret_cast<uint8_t*>(q);
  q += ((size_t)s.N + 15) & ~(size_t)15;
  L.obsrow = reinterpret_cast<uint8_t*>(q);
  q += ((size_t)s.N * s.Lc * s.E + 15) & ~(size_t)15;
  L.sink = reinterpret_cast<WT*>(q);
  return L;
}

// one env slot of the workgroup
template <int NT, int EPW, typename WT>
struct Ctx {
  static constexpr int LPE = NT / EPW;            // lanes per env
  static constexpr int KI = EPW == 1 ? 2 : 3;     // staged items per lane
  static constexpr int RPL = EPW == 1 ? 2 : 3;    // beams per lane per pass
  int sub;    // lane within the env
  int lane0;  // first lane of this env's slot within the wave
  int e;      // env index
  Lds<WT> L;
};

// broadcast lane (lane0 + i)'s value of v to the slot
template <int NT, int EPW, typename WT>
__device__ __forceinline__ int bcast(const Ctx<NT, EPW, WT>& C, int v, int i) {
  if constexpr (EPW == 1) return rdlane(v, i);
  else return __shfl(v, C.lane0 + i);
}

// ballot restricted to this env's slot (bit j = lane lane0 + j)
template <int NT, int EPW, typename WT>
__device__ __forceinline__ uint64_t slot_ballot(const Ctx<NT, EPW, WT>& C, bool p) {
  const uint64_t m = __ballot(p);
  if constexpr (EPW == 1) return m;
  else return (m >> C.lane0) & low_mask(Ctx<NT, EPW, WT>::LPE);
}

// staged (agent, row) items of this lane; raw HBM words stay in registers
// from stage to store
template <int KI, typename WT>
struct Items {
  int a[KI], gx[KI], oy[KI];
  uint64_t f0[KI], f1[KI], o0[KI], o1[KI], u0[KI], u1[KI];  // raw HBM words
  WT nf[KI], no[KI], nu[KI];                                  // new bits (window)
};

__device__ __forceinline__ bool row_in(const State& s, int gx) { return gx >= 0 && gx < s.Wp; }
__device__ __forceinline__ bool word0_in(const State& s, int gx, int oy) {
  const int w0 = oy >> 6;
  return row_in(s, gx) && w0 >= 0 && w0 < s.nw;
}
__device__ __forceinline__ bool word1_in(const State& s, int gx, int oy) {
  const int w1 = (oy >> 6) + 1;
  return row_in(s, gx) && w1 >= 0 && w1 < s.nw && (oy & 63) != 0;
}

// --------------------------------------------------------------------------
// stage: one round trip for every staged row (masks known zero after reset)
// --------------------------------------------------------------------------
template <int NT, int EPW, typename WT, int KI>
__device__ __forceinline__ void stage(const State& s, const Ctx<NT, EPW, WT>& C, bool load_masks,
                                      Items<KI, WT>& I) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int items = s.N * s.We;
  const size_t mw = (size_t)s.Wp * s.nw;
  const int g = L.sc->grid;
  const uint64_t* gn = s.grid_neg + (size_t)g * mw;
  const uint64_t* gp = s.grid_pos + (size_t)g * mw;
  const uint64_t wmask = low_mask(s.We);
  const bool square = s.sensor == 1;
  uint64_t n0[KI], n1[KI], p0[KI], p1[KI];
  // addresses first, then every load of the lane back to back with no
  // exec-mask branches (words outside the grid read index 0 and are
  // replaced below), so the whole stage is one memory round trip
  size_t i0[KI], i1[KI], fb[KI];
  bool in0[KI], in1[KI];
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    const bool it = idx < items;
    const int a = it ? udiv(idx, s.mg_We) : 0;
    const int r = idx - a * s.We;
    const int gx = L.x0[a] - s.H - 1 + r;
    const int oy = L.y0[a] - s.H - 1;
    I.a[k] = a;
    I.gx[k] = it ? gx : -1;
    I.oy[k] = oy;
    const int w0 = oy >> 6;
    in0[k] = it && word0_in(s, gx, oy);
    in1[k] = it && word1_in(s, gx, oy);
    const size_t rb = (size_t)(row_in(s, gx) ? gx : 0) * s.nw;
#if defined(MC_ABL) && MC_ABL == 7
    // timing ablation: word-planar addresses (word w of row x at w*Wp + x)
    i0[k] = in0[k] ? (size_t)w0 * s.Wp + (rb / s.nw) : 0;
    i1[k] = in1[k] ? (size_t)(w0 + 1) * s.Wp + (rb / s.nw) : 0;
#else
    i0[k] = in0[k] ? rb + w0 : 0;
    i1[k] = in1[k] ? rb + w0 + 1 : 0;
#endif
    fb[k] = ((size_t)C.e * s.N + a) * mw;
  }
  const size_t vb = (size_t)C.e * mw;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    n0[k] = gn[i0[k]];
    n1[k] = gn[i1[k]];
    if (load_masks) {
      I.f0[k] = s.freem[fb[k] + i0[k]];
      I.f1[k] = s.freem[fb[k] + i1[k]];
      I.o0[k] = s.obstm[fb[k] + i0[k]];
      I.o1[k] = s.obstm[fb[k] + i1[k]];
      I.u0[k] = s.vis[vb + i0[k]];
      I.u1[k] = s.vis[vb + i1[k]];
    }
    if (square) {
      p0[k] = gp[i0[k]];
      p1[k] = gp[i1[k]];
    }
  }
#ifdef MC_STAMPS
  STAMP(11);  // loads issued
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(12);  // loads landed
#endif
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    // outside the grid: blocked (isInBounds), no marks
    n0[k] = in0[k] ? n0[k] : ~0ull;
    n1[k] = in1[k] ? n1[k] : ~0ull;
    p0[k] = (square && in0[k]) ? p0[k] : 0;
    p1[k] = (square && in1[k]) ? p1[k] : 0;
    const bool m0 = load_masks && in0[k], m1 = load_masks && in1[k];
    I.f0[k] = m0 ? I.f0[k] : 0;
    I.o0[k] = m0 ? I.o0[k] : 0;
    I.u0[k] = m0 ? I.u0[k] : 0;
    I.f1[k] = m1 ? I.f1[k] : 0;
    I.o1[k] = m1 ? I.o1[k] : 0;
    I.u1[k] = m1 ? I.u1[k] : 0;
  }
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    if (idx < items) {
      const int off = I.oy[k] & 63;
      L.neg[idx] = (WT)(funnel(n0[k], n1[k], off) & wmask);
      L.pos[idx] = (WT)(funnel(p0[k], p1[k], off) & wmask);
      L.fold[idx] = (WT)(funnel(I.f0[k], I.f1[k], off) & wmask);
      L.oold[idx] = (WT)(funnel(I.o0[k], I.o1[k], off) & wmask);
      L.fp[idx] = 0;
      L.op[idx] = 0;
    }
  }
}

// --------------------------------------------------------------------------
// moves: updateRobotPos in robot order (dec_grid_rl.py:128-145, :171-204).
// Lane lane0+i = robot i of the slot.  Occupancy is the live position set: a
// robot may enter a cell vacated earlier in this step and is blocked by a
// higher-index robot that has not moved yet (:186,190-199,310).  The grid
// test reads the staged extended window (1 outside the grid = isInBounds).
// --------------------------------------------------------------------------
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void moves(const State& s, const Ctx<NT, EPW, WT>& C, double pen_unit) {
  const Lds<WT>& L = C.L;
  const int N = s.N;
  const bool live = C.sub < N;
  int x = live ? L.x0[C.sub] : INT32_MIN / 2;
  int y = live ? L.y0[C.sub] : INT32_MIN / 2;
  const int act = live ? (int)L.act[C.sub] : 255;
  const int dx = (act == 0) - (act == 2), dy = (act == 1) - (act == 3);
  int gblk = 1;
  if (live && act < 4) {
    const WT row = L.neg[C.sub * s.We + s.H + 1 + dx];
    gblk = (int)((row >> (s.H + 1 + dy)) & (WT)1);
  }
  const int tx = x + dx, ty = y + dy;
  double pen = 0.0;
  uint64_t moved = L.sc->moved;
  for (int i = 0; i < N; ++i) {
    const bool acts = bcast(C, act, i) <= 3;  // not 0..3: no updateRobotPos call, no penalty
    const int txi = bcast(C, tx, i), tyi = bcast(C, ty, i);
    const bool occ = slot_ballot(C, live && x == txi && y == tyi) != 0ull;
    const bool ok = acts && !bcast(C, gblk, i) && !occ;
    if (ok && C.sub == i) { x = txi; y = tyi; }
    if (ok) moved |= 1ull << i;
    if (acts && !ok) pen += pen_unit;  // reward += -collision_penalty (:203)
  }
  if (live) { L.x[C.sub] = x; L.y[C.sub] = y; }
  if (C.sub == 0) { L.sc->pen = pen; L.sc->moved = moved; }
}

// --------------------------------------------------------------------------
// lidar march (lidar.py:34-63), integer form.  The major coordinate moves
// exactly +-1 per step; the minor cell moves by msign at the steps flagged in
// the host-built beam_bits word for this (beam, start coordinate), which
// encodes the reference's float64 `+=` chain bit-exactly (mc_internal.h).
// Every cell of a beam lies within Chebyshev K <= H of the post-move robot,
// which is within 1 of the staged window's centre: no window check is
// needed (mc_set_beam_table rejects K > H).  RPL beams per lane advance in
// lock step; per step: one LDS read of the neg row and of the free row, and
// at most one ds_or (free mark, or obstacle mark that ends the beam), skipped
// when the free bit is already set.
// --------------------------------------------------------------------------
struct Ray {
  uint32_t bits;     // minor-move bit per step (K <= 31)
  int row, col;      // current window cell; LDS row index = agent base + row
  int drow, dcol;    // major step
  int mrow, mcol;    // minor step (when the step's bit is set)
  int K;
  bool live;
};

template <typename WT>
__device__ __forceinline__ Ray ray_init(const State& s, const Lds<WT>& L, int idx) {
  Ray R;
  R.live = idx < s.N * s.nbeams;
  const int a = R.live ? udiv(idx, s.mg_nb) : 0;
  const int b = R.live ? idx - a * s.nbeams : 0;
  const Beam bm = L.beams[b];
  const int xa = L.x[a], ya = L.y[a];
  R.row = a * s.We + xa - (L.x0[a] - s.H - 1);
  R.col = ya - (L.y0[a] - s.H - 1);
  const bool ax = bm.axis == 0;
  R.drow = ax ? bm.sign : 0;
  R.dcol = ax ? 0 : bm.sign;
  R.mrow = ax ? 0 : bm.msign;
  R.mcol = ax ? bm.msign : 0;
  R.K = R.live ? bm.K : -1;
  R.bits = R.live ? (uint32_t)s.beam_bits[(size_t)b * s.bcmax + (ax ? ya : xa)] : 0u;
  return R;
}

__device__ __forceinline__ void ray_advance(Ray& R, int k) {
  const bool mv = (R.bits >> k) & 1u;
  R.row += R.drow + (mv ? R.mrow : 0);
  R.col += R.dcol + (mv ? R.mcol : 0);
}

// Branch-free mark: every lane issues one ds_or per ray and step; a lane with
// nothing to mark ORs into its own sink word (no bank conflicts, no exec-mask
// branches).  Re-marking an already free cell is harmless (OR).
template <typename WT>
__device__ __forceinline__ void ray_mark(const Lds<WT>& L, Ray& R, int k, WT nrow, WT* sink) {
  const bool on = R.live && k <= R.K;
  const WT bit = (WT)1 << R.col;
  const bool hit = (nrow & bit) != 0;  // oc[int(cx), int(cy)] < 0: the beam ends here
#if defined(MC_ABL) && MC_ABL == 1
  lds_or(sink, bit);  // timing ablation: no marks
#else
  lds_or(on ? (hit ? L.op : L.fp) + R.row : sink, bit);
#endif
  R.live = on && !hit;
}

template <int NT, int EPW, typename WT>
__device__ __forceinline__ void sense(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  constexpr int RPL = Ctx<NT, EPW, WT>::RPL;
  const Lds<WT>& L = C.L;
  const int N = s.N, We = s.We, H = s.H;
  if (s.sensor == 0) {
    // step 0 of every beam is the robot's own (free) cell: mark it once
    for (int a = C.sub; a < N; a += LPE) {
      const int r0 = L.x[a] - (L.x0[a] - H - 1), c0 = L.y[a] - (L.y0[a] - H - 1);
      lds_or(&L.fp[a * We + r0], (WT)1 << c0);
    }
    const int total = N * s.nbeams;
    // lane l of a pass takes rays RPL*l .. RPL*l+RPL-1: within one ds_or the
    // lanes of an agent hold beams RPL apart, which mostly land in different
    // rows (fewer same-address LDS atomics than adjacent beams)
    for (int base = C.sub * RPL; base < total; base += RPL * LPE) {
      Ray q[RPL];
#pragma unroll
      for (int j = 0; j < RPL; ++j) {
        q[j] = ray_init<WT>(s, L, base + j);
        ray_advance(q[j], 0);
      }
      // wave-uniform trip count (every cell with k <= K <= beam_kmax <= H
      // lies inside the staged window)
      const int kmax = s.beam_kmax;
      WT* sink = L.sink + (threadIdx.x & 63);
      for (int k = 1; k <= kmax; ++k) {
        WT nr[RPL];
#pragma unroll
        for (int j = 0; j < RPL; ++j) nr[j] = L.neg[q[j].row];  // all row reads in flight
#pragma unroll
        for (int j = 0; j < RPL; ++j) {
          ray_mark<WT>(L, q[j], k, nr[j], sink);
          ray_advance(q[j], k);
        }
      }
    }
  } else {
    // window [x-r, x+r] x [y-r, y+r] clamped to the padded grid; the
    // reference overwrites it with clip(g,0,1) / clip(-g,0,1), which on a
    // static grid is an OR (every free bit comes from clip(g,0,1)).
    const int rr = s.sq_r;
    for (int idx = C.sub; idx < N * We; idx += LPE) {
      const int a = udiv(idx, s.mg_We), r = idx - a * We;
      const int ox = L.x0[a] - H - 1, oy = L.y0[a] - H - 1;
      const int gx = ox + r, xa = L.x[a], ya = L.y[a];
      WT f = 0, o = 0;
      if (gx >= xa - rr && gx <= xa + rr && gx >= 0 && gx < s.Wp) {
        int c0 = ya - rr - oy, c1 = ya + rr - oy;      // extended-window columns
        if (c0 < -oy) c0 = -oy;                          // grid column 0
        if (c1 > s.Lp - 1 - oy) c1 = s.Lp - 1 - oy;      // grid column Lp-1
        if (c1 >= c0) {
          const WT cm = (WT)(low_mask(c1 + 1) & ~low_mask(c0));
          f = L.pos[idx] & cm;
          o = L.neg[idx] & cm;
        }
      }
      L.fp[idx] = f;
      L.op[idx] = o;
    }
  }
}

// single_square_tool: only the robot's own cell becomes free (:233-234)
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void single_tool(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  for (int idx = C.sub; idx < s.N * s.We; idx += LPE) {
    const int a = udiv(idx, s.mg_We), r = idx - a * s.We;
    const int ox = L.x0[a] - s.H - 1, oy = L.y0[a] - s.H - 1;
    L.fp[idx] = (ox + r == L.x[a]) ? ((WT)1 << (L.y[a] - oy)) : (WT)0;
  }
}

// --------------------------------------------------------------------------
// merge (dec_grid_rl.py:232-256): newly set free bits per agent, and the
// union delta = cells some agent marked this step that were not yet visited,
// each counted at the lowest-index agent that marked it.
// --------------------------------------------------------------------------
template <int NT, int EPW, typename WT, int KI>
__device__ __forceinline__ void merge(const State& s, const Ctx<NT, EPW, WT>& C, Items<KI, WT>& I) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int items = s.N * s.We;
  const uint64_t wmask = low_mask(s.We);
  // EPW == 1: agent j's pre-move origin in lane j of every wave, broadcast by
  // v_readlane (N <= 64)
  const int jw = (int)(threadIdx.x & 63);
  const int jl = jw < s.N ? jw : 0;
  const int ax0 = L.x0[jl], ay0 = L.y0[jl];
  uint32_t cf = 0, cv = 0;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    I.nf[k] = I.no[k] = I.nu[k] = 0;
    if (idx < items) {
      const WT fp = L.fp[idx], op = L.op[idx];
      I.nf[k] = fp & ~L.fold[idx];
      I.no[k] = op & ~L.oold[idx];
      cf += popc(I.nf[k]);
      const int a = I.a[k], gx = I.gx[k], oy = I.oy[k];
      WT cand = fp & ~(WT)(funnel(I.u0[k], I.u1[k], oy & 63) & wmask);
#if defined(MC_ABL) && MC_ABL == 4
      for (int b = 0; b < 0; ++b) {  // timing ablation: no dedup
#else
      for (int b = 0; b < a; ++b) {  // marks of lower-index agents at these cells
#endif
        int xb, yb;
        if constexpr (EPW == 1) {
          xb = rdlane(ax0, b);
          yb = rdlane(ay0, b);
        } else {
          xb = L.x0[b];
          yb = L.y0[b];
        }
        const int rb = gx - (xb - s.H - 1);
        const int d = (yb - s.H - 1) - oy;  // column shift b -> a (|d| < We to overlap)
        if ((unsigned)rb < (unsigned)s.We && d > -s.We && d < s.We) {
          const WT pb = L.fp[b * s.We + rb];
          cand &= ~(d >= 0 ? (WT)(pb << d) : (WT)(pb >> -d));
        }
      }
      I.nu[k] = cand;
      cv += popc(cand);
    }
  }
  if (cf) atomicAdd(&L.sc->cnt_free, cf);
  if (cv) atomicAdd(&L.sc->cnt_vis, cv);
}

// after merge: fold |= fp (obs crops read the post-step maps)
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void fold_marks(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  for (int idx = C.sub; idx < s.N * s.We; idx += LPE) {
    C.L.fold[idx] |= C.L.fp[idx];
    C.L.oold[idx] |= C.L.op[idx];
  }
}

template <int NT, int EPW, typename WT, int KI>
__device__ __forceinline__ void store_words(const State& s, const Ctx<NT, EPW, WT>& C,
                                            const Items<KI, WT>& I) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const int items = s.N * s.We;
  const size_t mw = (size_t)s.Wp * s.nw;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    if (idx >= items) continue;
    const int gx = I.gx[k], oy = I.oy[k];
    if (!row_in(s, gx)) continue;
    const int w0 = oy >> 6, off = oy & 63;
    const bool in0 = word0_in(s, gx, oy), in1 = word1_in(s, gx, oy);
    const size_t rb = (size_t)gx * s.nw;
    const size_t fb = ((size_t)C.e * s.N + I.a[k]) * mw + rb;
    const uint64_t nf = I.nf[k], no = I.no[k], nu = I.nu[k];  // widened to the HBM word
    if (nf) {
      if (in0) s.freem[fb + w0] = I.f0[k] | (nf << off);
      if (in1) s.freem[fb + w0 + 1] = I.f1[k] | (nf >> (64 - off));
    }
    if (no) {
      if (in0) s.obstm[fb + w0] = I.o0[k] | (no << off);
      if (in1) s.obstm[fb + w0 + 1] = I.o1[k] | (no >> (64 - off));
    }
    if (nu) {  // agents' windows overlap: several lanes may add bits to one word
      unsigned long long* v = (unsigned long long*)(s.vis + (size_t)C.e * mw + rb);
      if (in0 && (nu << off)) atomicOr(v + w0, nu << off);
      if (in1 && (nu >> (64 - off))) atomicOr(v + w0 + 1, nu >> (64 - off));
    }
  }
}

// --------------------------------------------------------------------------
// reset (dec_grid_rl.py:449-531) of the slot's env inside the launch: grid
// pick, start cells (injected, or Philox rejection draw with the reference's
// acceptance rule, :491-502), zeroed maps, initial observe() (reward
// discarded, :524).
// --------------------------------------------------------------------------
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void reset_env(const State& s, const Ctx<NT, EPW, WT>& C,
                                          const int32_t* inj_pos) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  constexpr int KI = Ctx<NT, EPW, WT>::KI;
  const Lds<WT>& L = C.L;
  const int N = s.N;
  const int e = C.e;
  if (C.sub == 0) {
    const uint32_t ep = s.episode[e] + 1u;
    s.episode[e] = ep;
    L.sc->ep = ep;
    if (s.grid_mode == 1) {
      const uint4 r = philox(s.seed, make_uint4(0xFFFFFFFFu, (uint32_t)e, ep, 0x67726964u));
      const int g = (int)bounded(r.x, (uint32_t)s.G);
      L.sc->grid = g;
      s.env_grid[e] = g;
    }
    L.sc->moved = 0;
    L.sc->cnt_free = 0;
    L.sc->cnt_vis = 0;
  }
  __syncthreads();
  const uint32_t ep = L.sc->ep;
  const int g = L.sc->grid;
  const size_t mw = (size_t)s.Wp * s.nw;
  {  // zero this env's maps (:505-514)
    uint64_t* f = s.freem + (size_t)e * N * mw;
    uint64_t* o = s.obstm + (size_t)e * N * mw;
    for (size_t i = C.sub; i < (size_t)N * mw; i += LPE) { f[i] = 0; o[i] = 0; }
    uint64_t* v = s.vis + (size_t)e * mw;
    for (size_t i = C.sub; i < mw; i += LPE) v[i] = 0;
  }
  if (inj_pos != nullptr) {
    if (C.sub < N) {
      const int x = inj_pos[((size_t)e * N + C.sub) * 2];
      const int y = inj_pos[((size_t)e * N + C.sub) * 2 + 1];
      bool bad = grid_blocked(s, g, x, y);
      for (int j = 0; j < C.sub; ++j)
        bad |= (inj_pos[((size_t)e * N + j) * 2] == x && inj_pos[((size_t)e * N + j) * 2 + 1] == y);
      if (bad) atomicOr(s.err, ERR_INJECT);
      L.x0[C.sub] = L.x[C.sub] = x;
      L.y0[C.sub] = L.y[C.sub] = y;
    }
  } else if (C.sub < 64) {
    // x = randint(W), y = randint(L); accept iff grid >= 0 and unoccupied;
    // candidates (Philox counter = candidate index) are consumed strictly in
    // draw order, CPR of them per round
    const int lane = C.sub;
    constexpr int CPR = LPE < 64 ? LPE : 64;
    int px = INT32_MIN / 2, py = INT32_MIN / 2, placed = 0;
    for (int round = 0; round < 1024 && placed < N; ++round) {
      const uint32_t k = (uint32_t)(round * CPR + lane);
      const uint4 r = philox(s.seed, make_uint4(k, (uint32_t)e, ep, 0x706c6163u));
      const int cx = (int)bounded(r.x, (uint32_t)s.Wp);
      const int cy = (int)bounded(r.y, (uint32_t)s.Lp);
      uint64_t okm = slot_ballot(C, !grid_blocked(s, g, cx, cy));
      while (okm && placed < N) {
        const int j = __ffsll((unsigned long long)okm) - 1;
        okm &= okm - 1;
        const int qx = bcast(C, cx, j), qy = bcast(C, cy, j);
        const bool clash = slot_ballot(C, lane < placed && px == qx && py == qy) != 0ull;
        if (!clash) {
          if (lane == placed) { px = qx; py = qy; }
          ++placed;
        }
      }
    }
    if (placed < N && lane == 0) atomicOr(s.err, ERR_PLACEMENT);
    if (lane < N) {
      L.x0[lane] = L.x[lane] = px;
      L.y0[lane] = L.y[lane] = py;
    }
  }
  // the zeroing stores must land before the window stores / atomics below
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  Items<KI, WT> I;
  stage<NT, EPW, WT, KI>(s, C, /*load_masks=*/false, I);
  __syncthreads();
  sense<NT, EPW, WT>(s, C);
  __syncthreads();
  if (s.sst) { single_tool<NT, EPW, WT>(s, C); __syncthreads(); }
  merge<NT, EPW, WT, KI>(s, C, I);
  __syncthreads();
  fold_marks<NT, EPW, WT>(s, C);
  store_words<NT, EPW, WT, KI>(s, C, I);
  __syncthreads();
  if (C.sub == 0) {
    s.free_cnt[e] = L.sc->cnt_free;
    s.vis_cnt[e] = L.sc->cnt_vis;
    s.currstep[e] = 0;
  }
}

// --------------------------------------------------------------------------
// obs (dec_grid_rl.py:312-372): layer 0 robot_pad, 1 own free, 2 own obst,
// E x E around each robot.  Each (agent, layer, row) becomes one E-bit byte
// in LDS; the uint8 output is then written as dwords.
// --------------------------------------------------------------------------
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void write_obs(const State& s, const Ctx<NT, EPW, WT>& C, uint8_t* obs_out) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int N = s.N, E = s.E, ego = s.ego, Lc = s.Lc, H = s.H;
  const uint64_t moved = L.sc->moved;
  const WT emask = wmask_of<WT>(E);
  for (int idx = C.sub; idx < N * Lc * E; idx += LPE) {
    const int a = udiv(idx, s.mg_LcE), rem = idx - a * (Lc * E);
    const int layer = udiv(rem, s.mg_E), r = rem - layer * E;
    const int xa = L.x[a], ya = L.y[a];
    WT bits = 0;
    if (layer == 0) {
      const int cx = xa - ego + r, cy0 = ya - ego;
      for (uint64_t m = moved; m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        const int dc = L.y[j] - cy0;
        if (L.x[j] == cx && dc >= 0 && dc < E) bits |= (WT)1 << dc;
      }
    } else if (layer <= 2) {
      const int er = xa - ego + r - (L.x0[a] - H - 1);
      const int ec = ya - ego - (L.y0[a] - H - 1);
      const WT row = (layer == 1 ? L.fold : L.oold)[a * s.We + er];
      bits = (row >> ec) & emask;
    }
    L.obsrow[idx] = (uint8_t)bits;
  }
  __syncthreads();
  const int total = N * Lc * E * E;
  uint8_t* dst = obs_out + (size_t)C.e * total;
  if ((total & 3) == 0) {
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
    for (int i = C.sub; i < total / 4; i += LPE) {
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int q = 4 * i + j;
        const int row = udiv(q, s.mg_E), col = q - row * E;
        v |= (uint32_t)((L.obsrow[row] >> col) & 1) << (8 * j);
      }
      d32[i] = v;
    }
  } else {
    for (int q = C.sub; q < total; q += LPE) {
      const int row = udiv(q, s.mg_E), col = q - row * E;
      dst[q] = (uint8_t)((L.obsrow[row] >> col) & 1);
    }
  }
}

// --------------------------------------------------------------------------
// the env kernel: EPW envs per workgroup
// --------------------------------------------------------------------------
template <int NT, int EPW, typename WT, class SH>
__global__ __launch_bounds__(NT) void env_kernel(State s_in, int mode, const uint8_t* __restrict__ actions,
                                                 const uint8_t* __restrict__ env_mask,
                                                 const int32_t* __restrict__ inj_pos,
                                                 double* __restrict__ reward_out,
                                                 uint8_t* __restrict__ done_out,
                                                 uint8_t* __restrict__ obs_out,
                                                 uint8_t* __restrict__ adj_out) {
  State s = s_in;
  specialize<SH>(s);
  using CtxT = Ctx<NT, EPW, WT>;
  constexpr int LPE = CtxT::LPE;
  constexpr int KI = CtxT::KI;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int N = s.N;
  CtxT C;
  const int slot = EPW == 1 ? 0 : tid / LPE;
  C.sub = EPW == 1 ? tid : tid - slot * LPE;
  C.lane0 = EPW == 1 ? 0 : slot * LPE;
  const int e_raw = blockIdx.x * EPW + slot;
  const bool valid = e_raw < s.B;  // a short last workgroup leaves a slot idle
  C.e = valid ? e_raw : s.B - 1;
  const size_t slot_lds =
      env_lds_bytes(s.N, s.We, s.sensor == 0 ? s.nbeams : 0, s.Lc, s.E, sizeof(WT));
  C.L = carve<WT>(smem + slot * slot_lds, s);
  const Lds<WT>& L = C.L;
  const int e = C.e;

  const bool is_step = mode == MODE_STEP;
  const bool sentinel = valid && is_step && actions[(size_t)e * N] == 255;
  const bool reset_req = valid && !is_step && (env_mask == nullptr || env_mask[e] != 0);
  const bool active = valid && is_step && !sentinel;

  STAMP(0);
  // ---- round trip 1: positions, actions, scalars, beam table ---------------
  if (C.sub < N) {
    const int2 p = reinterpret_cast<const int2*>(s.pos)[(size_t)e * N + C.sub];
    L.x0[C.sub] = L.x[C.sub] = p.x;
    L.y0[C.sub] = L.y[C.sub] = p.y;
    if (active) L.act[C.sub] = actions[(size_t)e * N + C.sub];
  }
  if (C.sub == 0) {
    const int g = s.env_grid[e];
    L.sc->grid = g;
    L.sc->moved = s.moved[e];
    L.sc->pen = 0.0;
    L.sc->cnt_free = 0;
    L.sc->cnt_vis = 0;
    L.sc->do_reset = 0;
    if (active) {
      L.sc->free_old = s.free_cnt[e];
      L.sc->vis_old = s.vis_cnt[e];
      L.sc->currstep = s.currstep[e];
      L.sc->done_thresh = s.done_thresh[e];
    }
  }
  if (s.sensor == 0)
    for (int b = C.sub; b < s.nbeams; b += LPE) L.beams[b] = s.beams[b];
  __syncthreads();

  if (active) {
    STAMP(1);
    Items<KI, WT> I;
#if defined(MC_ABL) && MC_ABL == 6
    stage<NT, EPW, WT, KI>(s, C, false, I);  // timing ablation: grid words only
#else
    stage<NT, EPW, WT, KI>(s, C, true, I);  // ---- round trip 2 ----
#endif
    if (C.sub == 0) L.sc->numfree = s.numfree[L.sc->grid];
    __syncthreads();
    STAMP(2);
    if (C.sub < 64) moves<NT, EPW, WT>(s, C, -s.pen);
    __syncthreads();
    STAMP(3);
#if !(defined(MC_ABL) && MC_ABL == 3)
    sense<NT, EPW, WT>(s, C);
#endif
    __syncthreads();
    STAMP(4);
    if (s.sst) { single_tool<NT, EPW, WT>(s, C); __syncthreads(); }
    merge<NT, EPW, WT, KI>(s, C, I);
    __syncthreads();
    STAMP(5);
    if (C.sub == 0) {
      Scal* c = L.sc;
      const uint32_t fc = c->free_old + c->cnt_free;
      const uint32_t vc = c->vis_old + c->cnt_vis;
      const int cs = c->currstep + 1;                        // :154
      double r = c->pen;                                     // :120,132-145
      r += (double)c->cnt_vis;                               // :151,:256
      const double pc = (double)fc / (double)c->numfree;     // :552
      double dt = c->done_thresh;
      const double thr = (1.0 < dt) ? 1.0 : dt;              // min(done_thresh, 1)
      const bool covered = thr <= pc;
      if (covered) r += s.term;                              // :156-157
      bool done = false;
      if (covered) { dt += s.dincr; done = true; }           // :540-543
      else if (cs == s.maxsteps) done = true;                // :544-545
      reward_out[e] = r;
      done_out[e] = done ? 1 : 0;
      s.free_cnt[e] = fc;
      s.vis_cnt[e] = vc;
      s.currstep[e] = cs;
      s.done_thresh[e] = dt;
      c->do_reset = (done && s.auto_reset) ? 1 : 0;
    }
    __syncthreads();
    STAMP(6);
    if (!L.sc->do_reset) {
      fold_marks<NT, EPW, WT>(s, C);
      store_words<NT, EPW, WT, KI>(s, C, I);
      STAMP(7);
    } else {
      reset_env<NT, EPW, WT>(s, C, nullptr);  // the finished episode's words are not stored
    }
  } else if (reset_req) {
    reset_env<NT, EPW, WT>(s, C, inj_pos);
  } else {
    // sentinel step / env left out of a partial reset: obs of the current
    // state only (dec_grid_rl.py:104-107,160)
    Items<KI, WT> I;
    stage<NT, EPW, WT, KI>(s, C, true, I);
    if (C.sub == 0 && sentinel) {
      reward_out[e] = 0.0;
      done_out[e] = 1;
    }
  }
  __syncthreads();

  if (active || reset_req) {
    if (C.sub < N)
      reinterpret_cast<int2*>(s.pos)[(size_t)e * N + C.sub] = make_int2(L.x[C.sub], L.y[C.sub]);
    if (C.sub == 0) s.moved[e] = L.sc->moved;
  }
  STAMP(8);
#if !(defined(MC_ABL) && MC_ABL == 5)
  if (valid) write_obs<NT, EPW, WT>(s, C, obs_out);
#endif
  STAMP(9);
  if (valid && adj_out != nullptr) {  // updateCommmunicationGraph (:374-391)
    uint8_t* ad = adj_out + (size_t)e * N * N;
    for (int idx = C.sub; idx < N * N; idx += LPE) {
      const int i = idx / N, j = idx - i * N;
      const int dx = abs(L.x[i] - L.x[j]), dy = abs(L.y[i] - L.y[j]);
      ad[idx] = (max(dx, dy) <= s.comm_r) ? 1 : 0;
    }
  }
#ifdef MC_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
  STAMP(10);
}

// Envs per wave: two when an env fits 32 lanes (N <= 32, at most 3 staged
// rows and 3 beams per lane), else one env per workgroup of NT threads.
int env_pack(const State& s) {
  const int items = s.N * s.We;
  const int rays = s.sensor == 0 ? s.N * s.nbeams : 0;
  return (s.N <= 32 && items <= 3 * 32 && rays <= 3 * 32) ? 2 : 1;
}

// MARLCOV_SPECIALIZE=0 forces the generic (runtime-shape) kernels (A/B tests)
static bool getenv_spec() {
  static const bool on = [] {
    const char* v = getenv("MARLCOV_SPECIALIZE");
    return !(v && v[0] == '0');
  }();
  return on;
}

hipError_t launch_env(const State& s, int mode, const uint8_t* actions, const uint8_t* env_mask,
                      const int32_t* inj_pos, double* reward, uint8_t* done, uint8_t* obs,
                      uint8_t* adj, int nt, int epw, hipStream_t stream) {
  const bool narrow = s.We <= 32;
  const size_t slot_lds = env_lds_bytes(s.N, s.We, s.sensor == 0 ? s.nbeams : 0, s.Lc, s.E,
                                        narrow ? 4 : 8);
#define MC_LAUNCH_SH(T, P, W, SH)                                                               \
  hipLaunchKernelGGL((env_kernel<T, P, W, SH>), dim3((s.B + (P)-1) / (P)), dim3(T),              \
                     slot_lds * (P), stream, s, mode, actions, env_mask, inj_pos, reward, done,    \
                     obs, adj)
#define MC_LAUNCH(T, P, W) MC_LAUNCH_SH(T, P, W, Dynamic)
  using Dynamic = Shape<0, 0, 0, 0, 0>;
  using ShapeC2 = Shape<4, 10, 21, 2, 10>;  // the bench workload
  const bool spec_ok = getenv_spec();
  if (epw == 2) {
    if (narrow && spec_ok && ShapeC2::matches(s)) MC_LAUNCH_SH(64, 2, uint32_t, ShapeC2);
    else if (narrow) MC_LAUNCH(64, 2, uint32_t);
    else MC_LAUNCH(64, 2, uint64_t);
  } else if (narrow) {
    switch (nt) {
      case 64: MC_LAUNCH(64, 1, uint32_t); break;
      case 128: MC_LAUNCH(128, 1, uint32_t); break;
      case 256: MC_LAUNCH(256, 1, uint32_t); break;
      case 512: MC_LAUNCH(512, 1, uint32_t); break;
      default: MC_LAUNCH(1024, 1, uint32_t); break;
    }
  } else {
    switch (nt) {
      case 64: MC_LAUNCH(64, 1, uint64_t); break;
      case 128: MC_LAUNCH(128, 1, uint64_t); break;
      case 256: MC_LAUNCH(256, 1, uint64_t); break;
      case 512: MC_LAUNCH(512, 1, uint64_t); break;
      default: MC_LAUNCH(1024, 1, uint64_t); break;
    }
  }
#undef MC_LAUNCH_SH
#undef MC_LAUNCH
  return hipGetLastError();
}

}  // namespace mc
