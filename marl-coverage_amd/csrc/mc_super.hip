// mc_super.hip — batched SuperGridRL, the centralized fully observed env
// (Environments/super_grid_rl.py:18-463), and its
// extern "C" entry points (include/marlcov.h, mc_sg_*).
//
// Per step (mc_sg_step), two kernels on the caller's stream:
//   sg_step_kernel  one wave per env: scan order (:108-129), sequential moves
//                   with live occupancy (:121-174), the square sense windows
//                   in robot order with the reference's per-slot float64
//                   reward folds (:177-201), motion penalty (:203-208,
//                   227-243), np.sum of the slots (pairwise, :214), terminal
//                   reward and done (:215-223, 401-421), and the incremental
//                   update of the registered state planes (robot cells, the
//                   sensed windows of the obstacle / _free layers);
//   sg_dist_kernel  one workgroup per env: get_distance_map (:281-303) of the
//                   post-step _free map — exact L1 distance of every cell to
//                   the nearest cell with _free != 0, separable: a row pass
//                   (distance along the row) then a column pass (down/up
//                   min-plus sweeps), then 1 - d / max(d) in float32 into the
//                   dist layer.  That layer is also the NEXT step's pre-move
//                   distance_map (:117-118): _free does not change between
//                   get_state and the next get_distance_map, so the step
//                   kernel reads its dist terms from it (no second transform).
// Maps are row bitboards: uint64 [W][RW], RW = ceil(L/64); bits >= L of a
// row's last word are always 0.
//
// The transform's OpenCV semantics follow the oracle's SciPy restatement
// (oracle/super_ref.py): exact L1; with no source cell at all (an obstacle-
// free grid fully covered) d is -1 everywhere, so the layer is 2.0 — parity
// vs real cv2 unpinned.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "marlcov.h"
#include "mc_device.h"

namespace mc {
void set_last_error(const char* msg);
}

namespace mcs {

using mc::bounded;
using mc::dist_value;
using mc::low_mask;
using mc::philox;

enum : uint32_t { ERR_PLACEMENT = 1u << 2, ERR_INJECT = 1u << 3, ERR_KEY = 1u << 4 };
constexpr int kMaxAgents = 64;
constexpr int kMaxRadius = 15;   // a window row (2r+1 cells) fits 32 bits
constexpr int kMaxSide = 4096;
constexpr int kEnvsPerBlock = 4; // step / reset kernels: one wave per env
constexpr int kInfD = 0xFFFF;    // "no source" in the u16 distance planes
constexpr size_t kLdsLimit = 64 * 1024;

struct SState {
  int B, N, W, L, G, RW, r, P;
  double pen, fpen, term, dincr;
  int dist, scan, maxsteps, auto_reset, grid_mode;
  int dist_full;   // MARLCOV_SG_FULL_DIST=1: rewrite the whole distance layer every step
  int32_t* dist_M; // [B] max(d) of the layer as last written (-1 unknown, -2 no source)
  double* ep_pc;   // [B] episode record at done (before an auto-reset): percent_covered()
  int32_t* ep_len; // [B] ... and _currstep
  uint32_t mg_L;  // floor(i / L) == umulhi(i, mg_L) (L >= 2)
  uint64_t seed;
  uint32_t env0, grid0;   // global ids of env 0 / pool grid 0 (mc_sg_config)
  const uint64_t* gneg;   // [G][W][RW] grid < 0
  const uint64_t* gpos;   // [G][W][RW] grid > 0
  const int32_t* numpos;  // [G] count_nonzero(grid > 0)
  int32_t* env_grid;      // [B]
  int32_t* pos;           // [B][N][2]
  uint64_t* cov;          // [B][W][RW] sensed cells (_free == 0)
  uint64_t* obst;         // [B][W][RW] _observed_obstacles
  uint32_t* cov_cnt;      // [B] count_nonzero(_free < 1)
  int32_t* currstep;      // [B]
  double* done_thresh;    // [B]
  int32_t* a_prev;        // [B] (-1 = None)
  uint32_t* episode;      // [B]
  uint8_t* full;          // [B] state planes need a full rewrite
  uint32_t* err;
  uint8_t* planes;        // caller: [B][P+2][W][L]
  float* dist_plane;      // caller: [B][W][L]
  uint16_t* scratch;      // [B][W][pitch] distance planes when they exceed LDS
};

__device__ __forceinline__ int div_L(const SState& s, int i) {
  return s.L == 1 ? i : (int)__umulhi((uint32_t)i, s.mg_L);
}

__device__ __forceinline__ bool bit_at(const uint64_t* map, int RW, int x, int y) {
  return (map[(size_t)x * RW + (y >> 6)] >> (y & 63)) & 1ull;
}

// bits [c0, c0 + 32) of a row (c0 may be negative; bit b = cell c0 + b)
__device__ __forceinline__ uint32_t row_field(const uint64_t* row, int RW, int c0) {
  const int w0 = c0 >> 6, sh = c0 & 63;  // arithmetic shift: floor
  const uint64_t a = (w0 >= 0 && w0 < RW) ? row[w0] : 0ull;
  const uint64_t b = (w0 + 1 >= 0 && w0 + 1 < RW) ? row[w0 + 1] : 0ull;
  return (uint32_t)(sh ? (a >> sh) | (b << (64 - sh)) : a);
}

// OR field f (bit b = cell c0 + b; only in-row bits set) into a row
__device__ __forceinline__ void or_field(uint64_t* row, int RW, int c0, uint32_t f) {
  if (!f) return;
  const int w0 = c0 >> 6, sh = c0 & 63;
  const uint64_t F = f;
  const uint64_t lo = F << sh, hi = sh ? F >> (64 - sh) : 0ull;
  if (w0 >= 0 && lo) atomicOr((unsigned long long*)&row[w0], (unsigned long long)lo);
  if (w0 + 1 < RW && hi) atomicOr((unsigned long long*)&row[w0 + 1], (unsigned long long)hi);
}

__device__ __forceinline__ uint32_t mask32(int lo, int hi) {  // bits [lo, hi), 0 <= lo, hi <= 32
  if (hi <= lo) return 0u;
  const uint32_t h = hi >= 32 ? 0xFFFFFFFFu : ((1u << hi) - 1u);
  return h & ~((1u << lo) - 1u);
}

// numpy's pairwise float64 sum of a contiguous array (n <= 128): what
// np.sum(reward) computes at super_grid_rl.py:214
__device__ double np_pairwise_sum(const double* a, int n) {
  if (n < 8) {
    double res = -0.0;
    for (int i = 0; i < n; ++i) res += a[i];
    return res;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

__device__ __forceinline__ int wave_sum(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// --------------------------------------------------------------------------
// reset (:343-399) of env e by one wave: grid pick, zeroed maps, start cells
// (injected, or Philox candidates x = randint(W), y = randint(L) consumed in
// draw order with the reference's acceptance rule grid >= 0 and unoccupied,
// :378-388).  _done_thresh and a_prev are kept (the reference never resets
// them).  The state planes are flagged for a full rewrite.
// --------------------------------------------------------------------------
__device__ void sg_reset_env(const SState& s, int e, int lane, const int32_t* inj) {
  const int N = s.N;
  const uint32_t ep = s.episode[e] + 1u;
  int g = s.env_grid[e];
  if (s.grid_mode == 1) {
    const uint4 r = philox(s.seed, make_uint4(0xFFFFFFFFu, s.env0 + (uint32_t)e, ep, 0x53677264u));
    g = (int)bounded(r.x, (uint32_t)s.G);
  }
  const size_t mw = (size_t)s.W * s.RW;
  uint64_t* cov = s.cov + (size_t)e * mw;
  uint64_t* obst = s.obst + (size_t)e * mw;
  for (size_t i = lane; i < mw; i += 64) {
    cov[i] = 0ull;
    obst[i] = 0ull;
  }
  const uint64_t* gneg = s.gneg + (size_t)g * mw;
  int px = -1, py = -1;
  if (inj != nullptr) {
    if (lane < N) {
      px = inj[((size_t)e * N + lane) * 2];
      py = inj[((size_t)e * N + lane) * 2 + 1];
      bool bad = px < 0 || py < 0 || px >= s.W || py >= s.L || bit_at(gneg, s.RW, px, py);
      for (int j = 0; j < lane; ++j)
        bad |= inj[((size_t)e * N + j) * 2] == px && inj[((size_t)e * N + j) * 2 + 1] == py;
      if (bad) atomicOr(s.err, ERR_INJECT);
    }
  } else {
    int placed = 0;
    for (int round = 0; round < 4096 && placed < N; ++round) {
      const uint32_t k = (uint32_t)(round * 64 + lane);
      const uint4 r = philox(s.seed, make_uint4(k, s.env0 + (uint32_t)e, ep, 0x53706c63u));
      const int cx = (int)bounded(r.x, (uint32_t)s.W);
      const int cy = (int)bounded(r.y, (uint32_t)s.L);
      uint64_t okm = __ballot(!bit_at(gneg, s.RW, cx, cy));
      while (okm && placed < N) {
        const int j = __ffsll((unsigned long long)okm) - 1;
        okm &= okm - 1;
        const int qx = __shfl(cx, j), qy = __shfl(cy, j);
        const bool clash = __ballot(lane < placed && px == qx && py == qy) != 0ull;
        if (!clash) {
          if (lane == placed) {
            px = qx;
            py = qy;
          }
          ++placed;
        }
      }
    }
    if (placed < N && lane == 0) atomicOr(s.err, ERR_PLACEMENT);
  }
  if (lane < N) {
    s.pos[((size_t)e * N + lane) * 2] = px;
    s.pos[((size_t)e * N + lane) * 2 + 1] = py;
  }
  if (lane == 0) {
    s.episode[e] = ep;
    s.env_grid[e] = g;
    s.cov_cnt[e] = 0;
    s.currstep[e] = 0;
    s.full[e] = 1;
  }
}

__global__ __launch_bounds__(256) void sg_reset_kernel(SState s, const uint8_t* __restrict__ mask,
                                                       const int32_t* __restrict__ inj) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * kEnvsPerBlock + (threadIdx.x >> 6);
  if (e >= s.B) return;
  if (mask != nullptr && mask[e] == 0) return;
  sg_reset_env(s, e, lane, inj);
}

// --------------------------------------------------------------------------
// SuperGridRL.step (:74-225).  GPW envs per wave: the wave's lanes form GPW
// groups of NG = 64 / GPW lanes, lane li of group grp = robot li of env
// (wave * GPW + grp) (N <= NG).  Cross-lane steps (occupancy ballots, robot
// broadcasts, the count sum) stay inside a group; the few envs of a wave that
// finish an episode are then reset one after another by the whole wave.
// With N = 4, GPW = 16 fills every lane: one wave does what 16 did.
// --------------------------------------------------------------------------
// R >= 0: senseradius R at compile time — the window of every plane around
// the PRE-move cell, extended by the one cell a move can shift it, is loaded
// in a single round together with the target's dist value, and the post-move
// window comes from registers (one load round instead of one per window row,
// twice).  R < 0: any radius, rows loaded as the loops reach them.
template <int R, int GPW>
__global__ __launch_bounds__(256) void sg_step_kernel(SState s, const uint8_t* __restrict__ actions,
                                                      const int32_t* __restrict__ quot,
                                                      double* __restrict__ reward,
                                                      uint8_t* __restrict__ done) {
  constexpr int NG = 64 / GPW;  // lanes per env
  __shared__ double s_v[kEnvsPerBlock * GPW][NG];
  __shared__ int s_x[kEnvsPerBlock * GPW][NG], s_y[kEnvsPerBlock * GPW][NG];
  const int lane = threadIdx.x & 63;
  const int grp = GPW == 1 ? 0 : lane / NG, li = GPW == 1 ? lane : lane & (NG - 1), gb = grp * NG;
  const int slot_env = (threadIdx.x >> 6) * GPW + grp;  // env slot within the block
  const int e_raw = blockIdx.x * (kEnvsPerBlock * GPW) + slot_env;
  const bool valid = e_raw < s.B;
  const int e = valid ? e_raw : s.B - 1;
  // group-local ballot (bit j = lane li == j of this env) and broadcast
  auto gballot = [&](bool p) -> uint64_t {
    const uint64_t m = __ballot(p);
    return GPW == 1 ? m : (m >> gb) & low_mask(NG);
  };
  auto gshfl = [&](int v, int z) -> int { return __shfl(v, gb + z); };
  const int N = s.N, W = s.W, L = s.L, RW = s.RW, r = R >= 0 ? R : s.r;
  const bool me = valid && li < N;
  // every load that depends only on e is issued up front, unconditionally
  // (clamped indices: lanes without a robot read robot 0; absent quotients
  // read a_prev), and nothing is used before the one wait below, so the
  // compiler cannot split the round (it sank the cell load behind a wait on
  // the sentinel byte, and that behind the grid index)
  const size_t ri = (size_t)e * N + (li < N ? li : 0);
  const int2 p_raw = reinterpret_cast<const int2*>(s.pos)[ri];
  const int act_raw = actions[ri];
  const int act0 = actions[(size_t)e * N];
  const int g = s.env_grid[e];
  const int q_raw = (quot ? quot : s.a_prev)[e];
  const int ap = s.a_prev[e];
  const int cs0 = s.currstep[e];
  const uint32_t cc0 = s.cov_cnt[e];
  const double dt = s.done_thresh[e];
  asm volatile("" ::"v"(p_raw.x), "v"(p_raw.y), "v"(act_raw), "v"(act0), "v"(g), "v"(q_raw), "v"(ap),
               "v"(cs0), "v"(cc0), "v"(dt));
  const int my_act = me ? act_raw : 255;  // slot `li`'s action byte
  const int q = quot ? q_raw : 0;
  const int npos = s.numpos[g];  // used at the end only
  int dn = 0;
  if (act0 == 255) {  // action == -1 / None (:88-90); uniform over the group
    dn = 1;
    if (valid && li == 0) {
      reward[e] = 0.0;
      done[e] = 1;
      s.ep_pc[e] = (double)cc0 / (double)npos;
      s.ep_len[e] = cs0;
    }
  } else {
    const size_t mw = (size_t)W * RW;
    const uint64_t* gneg = s.gneg + (size_t)g * mw;
    const uint64_t* gpos = s.gpos + (size_t)g * mw;
    uint64_t* cov = s.cov + (size_t)e * mw;
    uint64_t* obst = s.obst + (size_t)e * mw;
    int x = me ? p_raw.x : -(1 << 20), y = me ? p_raw.y : -(1 << 20);
    const int x_old = x, y_old = y;
    // reward slot of robot `li` (r2c): its rank by x + y*W with scanning
    int slot = li;
    if (s.scan) {
      const int sc = x + y * W;
      int rank = 0;
      for (int j = 0; j < N; ++j) rank += gshfl(sc, j) < sc;
      slot = rank;
    }
    const int slot_act = gshfl(my_act, slot < NG ? slot : 0);
    const int u = me ? slot_act : 255;
    int tx = x, ty = y;
    if (u == 0) tx = x - 1;
    else if (u == 1) tx = x + 1;
    else if (u == 2) ty = y + 1;
    else if (u == 3) ty = y - 1;
    const bool inb = me && tx >= 0 && tx < W && ty >= 0 && ty < L;
    // pre-move distance_map[x, y] (:117-118, 139): the dist layer of the last
    // state (loaded whether or not the move succeeds: no wait on the grid)
    // (unconditional, clamped cell, any valid plane without dist_reward: it
    // joins the window's round)
    const float* dpl = s.dist ? s.dist_plane : reinterpret_cast<const float*>(s.gneg);
    const float dvr = dpl[s.dist && inb ? ((size_t)e * W + tx) * L + ty : 0];
    constexpr int NE = R >= 0 ? 2 * R + 3 : 1;  // extended window rows
    constexpr int kRowUnroll = R >= 0 ? 2 * R + 1 : 1;
    constexpr int kColUnroll = R >= 0 ? 2 * R + 1 : 1;
    uint32_t xn[NE], xp[NE], xc[NE];             // bit b = cell y - R - 1 + b
    bool gfree;
    if constexpr (R >= 0) {
      // every window word is loaded unconditionally from a clamped address
      // and masked afterwards: one round for all 6 * NE loads (predicated
      // loads made the compiler wait after every row: NE round trips)
      const int c0e = y - R - 1;
      const int w0 = c0e >> 6, sh = c0e & 63;  // arithmetic shift: floor
      const bool wa = w0 >= 0 && w0 < RW, wb = w0 + 1 >= 0 && w0 + 1 < RW;
      const size_t ia = wa ? (size_t)w0 : 0, ib = wb ? (size_t)(w0 + 1) : 0;
      // (the field's low 32 bits need only the low dword of the second word)
      uint64_t na[NE], pa[NE], ca[NE];
      uint32_t nb[NE], pb[NE], cb[NE];
      bool okr[NE];
      auto lo32 = [](const uint64_t* p) -> uint32_t { return *reinterpret_cast<const uint32_t*>(p); };
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        const int j = x - R - 1 + k;
        okr[k] = me && j >= 0 && j < W;
        const size_t ro = (size_t)(okr[k] ? j : 0) * RW;
        na[k] = gneg[ro + ia];
        nb[k] = lo32(gneg + ro + ib);
        pa[k] = gpos[ro + ia];
        pb[k] = lo32(gpos + ro + ib);
        ca[k] = cov[ro + ia];
        cb[k] = lo32(cov + ro + ib);
      }
      auto fld = [&](uint64_t a, uint32_t b, bool ok) -> uint32_t {
        const uint64_t A = (ok && wa) ? a : 0ull, Bw = (ok && wb) ? (uint64_t)b : 0ull;
        return (uint32_t)(sh ? (A >> sh) | (Bw << (64 - sh)) : A);
      };
      asm volatile("" ::"v"(na[NE - 1]), "v"(nb[NE - 1]), "v"(pa[NE - 1]), "v"(pb[NE - 1]), "v"(ca[NE - 1]),
                   "v"(cb[NE - 1]), "v"(dvr));  // the round's single wait
#pragma unroll
      for (int k = 0; k < NE; ++k) {
        xn[k] = fld(na[k], nb[k], okr[k]);
        xp[k] = fld(pa[k], pb[k], okr[k]);
        xc[k] = fld(ca[k], cb[k], okr[k]);
      }
      const int ddx = tx - x, ddy = ty - y;
      const uint32_t trow = ddx < 0 ? xn[R] : (ddx > 0 ? xn[R + 2] : xn[R + 1]);
      gfree = inb && !((trow >> (R + 1 + ddy)) & 1u);
    } else {
      gfree = inb && !bit_at(gneg, RW, tx, ty);
    }
    const double dv = (s.dist && inb && u < 4) ? (double)dvr : 0.0;
    double v = 0.0;
    for (int k = 0; k < N; ++k) {  // slot order; robot z = the one with slot k
      const int z = s.scan ? (__ffsll((unsigned long long)gballot(me && slot == k)) - 1) : k;
      const int zu = gshfl(u, z);
      const int zx = gshfl(tx, z), zy = gshfl(ty, z);
      const int zok = gshfl((int)gfree, z);
      const bool occ = gballot(me && x == zx && y == zy) != 0ull;
      if (zu < 4 && li == z) {  // not a move: nothing happens (no penalty)
        if (zok && !occ) {
          x = zx;
          y = zy;
          if (s.dist) v = v + dv;
        } else {
          v = v - s.pen;
        }
      }
    }
    if (me) {
      s_x[slot_env][li] = x;
      s_y[slot_env][li] = y;
    }
    wave_sync();

    // sense (:177-201): robot i's window, raster order; a cell with grid >= 0
    // is new (+grid) unless covered before this step or by a lower robot's
    // window, else -free_penalty; grid < 0 marks an observed obstacle.  Phase
    // A reads only; the map updates follow in phase B.
    const int n = 2 * r + 1;
    const int c0 = y - r;
    const uint32_t vm = mask32(max(0, -c0), min(n, L - c0));
    const int mdx = x - x_old, msh = 1 + (y - y_old);  // post-move window in the extended one
    // window row jj of plane `a`: from the staged registers (R >= 0) or HBM
    auto field = [&](const uint32_t* a, const uint64_t* plane, int jj, int j) -> uint32_t {
      if constexpr (R >= 0) {
        const uint32_t t = mdx < 0 ? a[jj] : (mdx > 0 ? a[jj + 2] : a[jj + 1]);
        return (t >> msh) & vm;
      } else {
        return row_field(plane + (size_t)j * RW, RW, c0) & vm;
      }
    };
    int cnt = 0;
    if (me) {
#pragma unroll kRowUnroll
      for (int jj = 0; jj < (R >= 0 ? 2 * R + 1 : n); ++jj) {
        const int j = x - r + jj;
        if (j < 0 || j >= W) continue;
        const uint32_t fneg = field(xn, gneg, jj, j);
        const uint32_t fpos = field(xp, gpos, jj, j);
        const uint32_t fcov = field(xc, cov, jj, j);
        uint32_t lower = 0;
        for (int m = 0; m < N; ++m) {  // uniform trip count; robots m < li count
          const int xm = s_x[slot_env][m], ym = s_y[slot_env][m];
          const uint32_t cm = mask32(max(0, ym - r - c0), min(n, ym + r + 1 - c0));
          lower |= (m < li && abs(j - xm) <= r) ? cm : 0u;
        }
        const uint32_t ge0 = vm & ~fneg;
        const uint32_t nw = ge0 & ~fcov & ~lower;
        cnt += __popc(nw);
        // raster fold, branch-free: v - fpen == v + (-fpen) in IEEE
        const double mfp = -s.fpen;
#pragma unroll kColUnroll
        for (int b = 0; b < (R >= 0 ? 2 * R + 1 : n); ++b) {
          const double t = ((nw >> b) & 1u) ? (((fpos >> b) & 1u) ? 1.0 : 0.0) : mfp;
          const double vt = v + t;
          v = ((ge0 >> b) & 1u) ? vt : v;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every read above is done
    // phase B: maps (idempotent ORs of the whole window) and state planes
    const size_t WL = (size_t)W * L;
    uint8_t* pl = s.planes + (size_t)e * (s.P + 2) * WL;
    if (me) {
      uint8_t* pl_obst = pl + (size_t)s.P * WL;
      uint8_t* pl_free = pl + (size_t)(s.P + 1) * WL;
#pragma unroll kRowUnroll
      for (int jj = 0; jj < (R >= 0 ? 2 * R + 1 : n); ++jj) {
        const int j = x - r + jj;
        if (j < 0 || j >= W) continue;
        const uint32_t fneg = field(xn, gneg, jj, j);
        const uint32_t ge0 = vm & ~fneg;
        // staged window: OR only the bits not covered before this step (covered
        // bits are cleared only by the reset below), so re-sensed rows cost no atomic
        if constexpr (R >= 0)
          or_field(cov + (size_t)j * RW, RW, c0, ge0 & ~field(xc, cov, jj, j));
        else
          or_field(cov + (size_t)j * RW, RW, c0, ge0);
        or_field(obst + (size_t)j * RW, RW, c0, fneg);
        uint8_t* row_o = pl_obst + (size_t)j * L + c0;
        uint8_t* row_f = pl_free + (size_t)j * L + c0;
        // staged window: a cell covered before this step already holds 0 in
        // _free (the layers track the bitboards, and a full rewrite follows any
        // reset / upload), so only new cells and obstacles are stored
        uint32_t st = vm;
        if constexpr (R >= 0) st = (ge0 & ~field(xc, cov, jj, j)) | fneg;
#pragma unroll kColUnroll
        for (int b = 0; b < (R >= 0 ? 2 * R + 1 : n); ++b) {  // obstacle -> 1 in layer P, else 0 in _free
          const bool ob = (fneg >> b) & 1u;
          uint8_t* dst = (ob ? row_o : row_f) + b;
          if ((st >> b) & 1u) *dst = ob ? 1 : 0;
        }
      }
    }
    // robot cells: clear the old one, set the new one.  With one shared layer
    // (use_scanning) a cell vacated by one robot may be entered by another in
    // the same step: that clear is skipped, so no store has to wait for
    // another (robots are distinct, so each cell gets one store at most)
    const bool moved = me && (x != x_old || y != y_old);
    const size_t lay = (size_t)(s.scan ? 0 : li) * WL;
    bool reoccupied = false;
    if (s.scan && me)
      for (int m = 0; m < N; ++m) reoccupied |= s_x[slot_env][m] == x_old && s_y[slot_env][m] == y_old;
    if (moved && !reoccupied) pl[lay + (size_t)x_old * L + y_old] = 0;
    if (moved) pl[lay + (size_t)x * L + y] = 1;

    // motion_penalty(a) on every slot (:203-208, 227-243): a is the quotient
    // left in `action` after the digit loop; a == inv(a) never holds
    if ((q < 0 || q >= 4) && valid && li == 0) atomicOr(s.err, ERR_KEY);
    v = v + ((q == ap) ? 0.0 : -1.0);
    if (me) {
      s_v[slot_env][slot] = v;
      s.pos[((size_t)e * N + li) * 2] = x;
      s.pos[((size_t)e * N + li) * 2 + 1] = y;
    }
#pragma unroll
    for (int o = NG / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);  // group sum
    wave_sync();
    if (valid && li == 0) {
      double total = np_pairwise_sum(s_v[slot_env], N);
      const int cs = cs0 + 1;
      const uint32_t cc = cc0 + (uint32_t)cnt;
      const double pc = (double)cc / (double)npos;
      const bool cond = (dt < 1.0 ? dt : 1.0) <= pc;  // min(_done_thresh, 1) <= percent_covered()
      if (cond) total = total + s.term;
      if (cond) s.done_thresh[e] = dt + s.dincr;  // done() (:408-411)
      dn = cond || (s.maxsteps > 0 && cs == s.maxsteps);
      s.a_prev[e] = q;
      s.currstep[e] = cs;
      s.cov_cnt[e] = cc;
      reward[e] = total;
      done[e] = (uint8_t)dn;
      if (dn) {  // the episode record (Utils/utils.py:138-141)
        s.ep_pc[e] = pc;
        s.ep_len[e] = cs;
      }
    }
  }
  // auto-reset: the wave's finished envs, one after another, each by every
  // lane of the wave (sg_reset_env draws 64 candidates per round)
  uint64_t rs = __ballot(s.auto_reset && valid && li == 0 && dn != 0);
  if (rs) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the step's map ORs land first
    const int e0 = blockIdx.x * (kEnvsPerBlock * GPW) + (int)(threadIdx.x >> 6) * GPW;
    for (; rs; rs &= rs - 1) {
      const int gj = (__ffsll((unsigned long long)rs) - 1) / NG;
      sg_reset_env(s, e0 + gj, lane, nullptr);
    }
  }
}

// --------------------------------------------------------------------------
// SuperGridRL.step with each robot's window rows spread over lanes (compiled
// radius R, at least 4 lanes per robot).  The group's lanes are robot-major:
// lane li = robot (li >> lgRL), row lane q = li & (RL - 1), RL = NG / P2(N)
// (P2: N rounded up to a power of two).  Every lane of a robot loads that
// robot's cell and action and replays the robot-order moves (the same values
// on all of them); row lane q senses window rows q, q + RL (n = 2R + 1 <= 7
// rows, so at most two), loading for each the three extended-window rows a
// move can bring into it.  The reference folds a robot's reward cells in
// raster order (float64, :177-201): each row lane publishes its rows' cell
// masks, and every lane of the robot runs the robot's whole fold from them.
// Same results as sg_step_kernel<R, GPW> (which takes one lane per robot).
// --------------------------------------------------------------------------
// DPP broadcasts inside a 16-lane row (one env of a GPW = 4 wave): lane L of
// the row (row_share), lane j of each quad (quad_perm), and a row sum into
// its lane 0 (row_shl steps; lanes shifted in from outside the row read 0)
template <int L>
__device__ __forceinline__ int row_share(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x150 | L, 0xF, 0xF, false); }
template <int L>
__device__ __forceinline__ double row_share_f64(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)row_share<L>((int)(uint32_t)b), hi = (uint32_t)row_share<L>((int)(uint32_t)(b >> 32));
  return __builtin_bit_cast(double, (uint64_t)lo | ((uint64_t)hi << 32));
}
template <int J>
__device__ __forceinline__ int quad_share(int v) {
  return __builtin_amdgcn_update_dpp(0, v, J | (J << 2) | (J << 4) | (J << 6), 0xF, 0xF, false);
}
__device__ __forceinline__ int row_sum_to_lane0(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x101, 0xF, 0xF, true);  // row_shl:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x102, 0xF, 0xF, true);  // row_shl:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x104, 0xF, 0xF, true);  // row_shl:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x108, 0xF, 0xF, true);  // row_shl:8
  return v;
}

template <int R, int GPW>
__global__ __launch_bounds__(256) void sg_step_rows(SState s, const uint8_t* __restrict__ actions,
                                                    const int32_t* __restrict__ quot,
                                                    double* __restrict__ reward,
                                                    uint8_t* __restrict__ done) {
  static_assert(R >= 1 && 2 * R + 1 <= 8, "compiled radius: a row's masks fit 8 bits");
  constexpr int NG = 64 / GPW;  // lanes per env
  constexpr int n = 2 * R + 1;  // window rows / columns
  constexpr int RPL = 2;        // window rows per lane (RL >= 4, n <= 7)
  __shared__ double s_v[kEnvsPerBlock * GPW][NG];
  __shared__ int s_x[kEnvsPerBlock * GPW][NG], s_y[kEnvsPerBlock * GPW][NG];
  const int lane = threadIdx.x & 63;
  const int grp = GPW == 1 ? 0 : lane / NG, li = GPW == 1 ? lane : lane & (NG - 1), gb = grp * NG;
  const int slot_env = (threadIdx.x >> 6) * GPW + grp;
  const int e_raw = blockIdx.x * (kEnvsPerBlock * GPW) + slot_env;
  const bool valid = e_raw < s.B;
  const int e = valid ? e_raw : s.B - 1;
  const int N = s.N, W = s.W, L = s.L, RW = s.RW;
  const int lgP2 = N <= 1 ? 0 : 32 - __clz(N - 1);
  const int lgRL = __builtin_ctz((unsigned)NG) - lgP2;  // launch_sg_step: RL >= 4
  const int RL = 1 << lgRL;
  const int i = li >> lgRL, q = li & (RL - 1);
  const bool me = valid && i < N;
  // one env per 16-lane row and one robot per quad, robots in slot order:
  // broadcasts by DPP instead of LDS shuffles
  const bool dpp = NG == 16 && RL == 4 && !s.scan;
  auto gballot = [&](bool p) -> uint64_t {
    const uint64_t m = __ballot(p);
    return GPW == 1 ? m : (m >> gb) & low_mask(NG);
  };
  auto gshfl = [&](int v, int z) -> int { return __shfl(v, gb + z); };
  auto rlane = [&](int robot) -> int { return robot << lgRL; };  // first lane of a robot
  // ---- round 1: every load that depends only on e (clamped indices) ----
  const size_t ri = (size_t)e * N + (i < N ? i : 0);
  const int2 p_raw = reinterpret_cast<const int2*>(s.pos)[ri];
  const int act_raw = actions[ri];
  const int act0 = actions[(size_t)e * N];
  const int g = s.env_grid[e];
  const int q_raw = (quot ? quot : s.a_prev)[e];
  const int ap = s.a_prev[e];
  const int cs0 = s.currstep[e];
  const uint32_t cc0 = s.cov_cnt[e];
  const double dt = s.done_thresh[e];
  asm volatile("" ::"v"(p_raw.x), "v"(p_raw.y), "v"(act_raw), "v"(act0), "v"(g), "v"(q_raw), "v"(ap),
               "v"(cs0), "v"(cc0), "v"(dt));
  const int my_act = me ? act_raw : 255;  // action byte i
  const int qt = quot ? q_raw : 0;
  const int npos = s.numpos[g];  // used at the end only
  int dn = 0;
  if (act0 == 255) {  // action == -1 / None (:88-90); uniform over the group
    dn = 1;
    if (valid && li == 0) {
      reward[e] = 0.0;
      done[e] = 1;
      s.ep_pc[e] = (double)cc0 / (double)npos;
      s.ep_len[e] = cs0;
    }
  } else {
    const size_t mw = (size_t)W * RW;
    const uint64_t* gneg = s.gneg + (size_t)g * mw;
    const uint64_t* gpos = s.gpos + (size_t)g * mw;
    uint64_t* cov = s.cov + (size_t)e * mw;
    uint64_t* obst = s.obst + (size_t)e * mw;
    int x = me ? p_raw.x : -(1 << 20), y = me ? p_raw.y : -(1 << 20);
    const int x_old = x, y_old = y;
    int slot = i;  // reward slot of robot i (r2c): its rank by x + y*W with scanning
    if (s.scan) {
      const int sc = x + y * W;
      int rank = 0;
      for (int j = 0; j < N; ++j) rank += gshfl(sc, rlane(j)) < sc;
      slot = rank;
    }
    // (without scanning slot = i: every lane of robot i holds its byte)
    const int slot_act = s.scan ? gshfl(my_act, rlane(slot < N ? slot : 0)) : my_act;
    const int u = me ? slot_act : 255;
    int tx = x, ty = y;
    if (u == 0) tx = x - 1;
    else if (u == 1) tx = x + 1;
    else if (u == 2) ty = y + 1;
    else if (u == 3) ty = y - 1;
    const bool inb = me && tx >= 0 && tx < W && ty >= 0 && ty < L;
    // ---- round 2: the target's grid word and dist value, and for each of
    // the lane's window rows the three extended rows (pre-move row x - R + jj
    // and its neighbours) of the three planes, all from clamped addresses ----
    const float* dpl = s.dist ? s.dist_plane : reinterpret_cast<const float*>(s.gneg);
    const float dvr = dpl[s.dist && inb ? ((size_t)e * W + tx) * L + ty : 0];
    const uint64_t tword = gneg[inb ? (size_t)tx * RW + (ty >> 6) : 0];
    const int c0e = y - R - 1;
    const int w0 = c0e >> 6, sh = c0e & 63;  // arithmetic shift: floor
    const bool wa = w0 >= 0 && w0 < RW, wb = w0 + 1 >= 0 && w0 + 1 < RW;
    const size_t ia = wa ? (size_t)w0 : 0, ib = wb ? (size_t)(w0 + 1) : 0;
    auto lo32 = [](const uint64_t* p) -> uint32_t { return *reinterpret_cast<const uint32_t*>(p); };
    uint64_t na[RPL][3], pa[RPL][3], ca[RPL][3];
    uint32_t nb[RPL][3], pb[RPL][3], cb[RPL][3];
    bool okr[RPL][3];
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int jj = q + k * RL;                // window row
        const int j = x - R - 1 + jj + t;         // extended row jj + t (pre-move frame)
        okr[k][t] = me && jj < n && j >= 0 && j < W;
        const size_t ro = (size_t)(okr[k][t] ? j : 0) * RW;
        na[k][t] = gneg[ro + ia];
        nb[k][t] = lo32(gneg + ro + ib);
        pa[k][t] = gpos[ro + ia];
        pb[k][t] = lo32(gpos + ro + ib);
        ca[k][t] = cov[ro + ia];
        cb[k][t] = lo32(cov + ro + ib);
      }
    }
    asm volatile("" ::"v"(na[RPL - 1][2]), "v"(nb[RPL - 1][2]), "v"(pa[RPL - 1][2]), "v"(pb[RPL - 1][2]),
                 "v"(ca[RPL - 1][2]), "v"(cb[RPL - 1][2]), "v"(dvr), "v"(tword));  // the round's one wait
    const bool gfree = inb && !((tword >> (ty & 63)) & 1ull);
    const double dv = (s.dist && inb && u < 4) ? (double)dvr : 0.0;
    // ---- moves in slot order (:121-174), replayed by every lane of a robot ----
    double v = 0.0;
    auto move = [&](int z, int zu, int zx, int zy, int zok) {
      const bool occ = gballot(me && x == zx && y == zy) != 0ull;
      if (zu < 4 && i == z) {  // not a move: nothing happens (no penalty)
        if (zok && !occ) {
          x = zx;
          y = zy;
          if (s.dist) v = v + dv;
        } else {
          v = v - s.pen;
        }
      }
    };
    if constexpr (NG == 16) {
      if (dpp) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (k < N) {
            const int zl = 4 * k;
            switch (k) {
              case 0: move(0, row_share<0>(u), row_share<0>(tx), row_share<0>(ty), row_share<0>((int)gfree)); break;
              case 1: move(1, row_share<4>(u), row_share<4>(tx), row_share<4>(ty), row_share<4>((int)gfree)); break;
              case 2: move(2, row_share<8>(u), row_share<8>(tx), row_share<8>(ty), row_share<8>((int)gfree)); break;
              default: move(3, row_share<12>(u), row_share<12>(tx), row_share<12>(ty), row_share<12>((int)gfree)); break;
            }
            (void)zl;
          }
        }
      }
    }
    if (!dpp) {
      for (int k = 0; k < N; ++k) {  // robot z = the one with slot k
        const int z = s.scan ? ((__ffsll((unsigned long long)gballot(me && q == 0 && slot == k)) - 1) >> lgRL) : k;
        const int zl = rlane(z);
        move(z, gshfl(u, zl), gshfl(tx, zl), gshfl(ty, zl), gshfl((int)gfree, zl));
      }
      if (me && q == 0) {
        s_x[slot_env][i] = x;
        s_y[slot_env][i] = y;
      }
      wave_sync();
    }
    // ---- sense (:177-201): the lane's rows; a cell with grid >= 0 is new
    // unless covered before this step or inside a lower robot's window ----
    const int c0 = y - R;
    const uint32_t vm = mask32(max(0, -c0), min(n, L - c0));
    const int mdx = x - x_old, msh = 1 + (y - y_old);  // post-move window in the extended one
    auto fld = [&](uint64_t a, uint32_t b, bool ok) -> uint32_t {
      const uint64_t A = (ok && wa) ? a : 0ull, Bw = (ok && wb) ? (uint64_t)b : 0ull;
      return (uint32_t)(sh ? (A >> sh) | (Bw << (64 - sh)) : A);
    };
    uint32_t rneg[RPL], rpos[RPL], rcov[RPL], rnw[RPL], rge[RPL];
    bool rin[RPL];
    int cnt = 0;
    // lower robots' window columns (relative to c0) and rows, once per robot
    // (at most NG / 4 robots: RL >= 4)
    constexpr int NMAX = NG / 4;
    uint32_t lcm[NMAX];
    int lxm[NMAX];
#pragma unroll
    for (int m = 0; m < NMAX; ++m) {
      const bool lo = m < N && m < i;
      int xm, ym;
      if (NG == 16 && dpp) {  // robot m's post-move cell from its quad
        xm = m == 0 ? row_share<0>(x) : (m == 1 ? row_share<4>(x) : (m == 2 ? row_share<8>(x) : row_share<12>(x)));
        ym = m == 0 ? row_share<0>(y) : (m == 1 ? row_share<4>(y) : (m == 2 ? row_share<8>(y) : row_share<12>(y)));
      } else {
        xm = s_x[slot_env][m < N ? m : 0];
        ym = s_y[slot_env][m < N ? m : 0];
      }
      lcm[m] = lo ? mask32(max(0, ym - R - c0), min(n, ym + R + 1 - c0)) : 0u;
      lxm[m] = xm;
    }
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      const int jj = q + k * RL;
      const int j = x - R + jj;
      const int t = 1 + mdx;  // post-move row jj is extended row jj + 1 + mdx
      const uint64_t an = t == 0 ? na[k][0] : (t == 1 ? na[k][1] : na[k][2]);
      const uint32_t bn = t == 0 ? nb[k][0] : (t == 1 ? nb[k][1] : nb[k][2]);
      const uint64_t ap_ = t == 0 ? pa[k][0] : (t == 1 ? pa[k][1] : pa[k][2]);
      const uint32_t bp = t == 0 ? pb[k][0] : (t == 1 ? pb[k][1] : pb[k][2]);
      const uint64_t ac = t == 0 ? ca[k][0] : (t == 1 ? ca[k][1] : ca[k][2]);
      const uint32_t bc = t == 0 ? cb[k][0] : (t == 1 ? cb[k][1] : cb[k][2]);
      const bool ok = t == 0 ? okr[k][0] : (t == 1 ? okr[k][1] : okr[k][2]);
      rin[k] = me && jj < n && j >= 0 && j < W;
      rneg[k] = (fld(an, bn, ok) >> msh) & vm;
      rpos[k] = (fld(ap_, bp, ok) >> msh) & vm;
      rcov[k] = (fld(ac, bc, ok) >> msh) & vm;
      uint32_t lower = 0;
#pragma unroll
      for (int m = 0; m < NMAX; ++m) lower |= (abs(j - lxm[m]) <= R) ? lcm[m] : 0u;  // robots m < i
      rge[k] = rin[k] ? (vm & ~rneg[k]) : 0u;
      rnw[k] = rge[k] & ~rcov[k] & ~lower;
      cnt += __popc(rnw[k]);
    }
    // the lane's rows' masks (nw, ge0, fpos: one byte each), row k at bits
    // 24k..; the robot's row jj is in lane jj & (RL - 1), slot jj >> lgRL
    uint64_t pub64 = 0;
#pragma unroll
    for (int k = 0; k < RPL; ++k)
      pub64 |= (uint64_t)(rnw[k] | (rge[k] << 8) | ((rpos[k] & 0xFFu) << 16)) << (24 * k);
    const double mfp = -s.fpen;
#pragma unroll
    for (int jj = 0; jj < n; ++jj) {
      uint32_t lo, hi;
      if (NG == 16 && dpp) {  // row lane jj & 3 of this robot's quad
        const int pl = (int)(uint32_t)pub64, ph = (int)(uint32_t)(pub64 >> 32);
        switch (jj & 3) {
          case 0: lo = (uint32_t)quad_share<0>(pl); hi = (uint32_t)quad_share<0>(ph); break;
          case 1: lo = (uint32_t)quad_share<1>(pl); hi = (uint32_t)quad_share<1>(ph); break;
          case 2: lo = (uint32_t)quad_share<2>(pl); hi = (uint32_t)quad_share<2>(ph); break;
          default: lo = (uint32_t)quad_share<3>(pl); hi = (uint32_t)quad_share<3>(ph); break;
        }
      } else {
        const int src = gb + rlane(i < N ? i : 0) + (jj & (RL - 1));
        lo = (uint32_t)__shfl((int)(uint32_t)pub64, src);
        hi = (uint32_t)__shfl((int)(uint32_t)(pub64 >> 32), src);
      }
      const uint64_t w = (uint64_t)lo | ((uint64_t)hi << 32);
      const uint32_t row = (uint32_t)(w >> (24 * (jj >> lgRL)));
      const uint32_t nw = row & 0xFFu, ge0 = (row >> 8) & 0xFFu, fpos = (row >> 16) & 0xFFu;
      // raster fold, branch-free: v - fpen == v + (-fpen) in IEEE
#pragma unroll
      for (int b = 0; b < n; ++b) {
        const double tv = ((nw >> b) & 1u) ? (((fpos >> b) & 1u) ? 1.0 : 0.0) : mfp;
        const double vt = v + tv;
        v = ((ge0 >> b) & 1u) ? vt : v;
      }
    }
    // ---- phase B: maps and state planes of the lane's rows ----
    const size_t WL = (size_t)W * L;
    uint8_t* pl = s.planes + (size_t)e * (s.P + 2) * WL;
    uint8_t* pl_obst = pl + (size_t)s.P * WL;
    uint8_t* pl_free = pl + (size_t)(s.P + 1) * WL;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
      if (!rin[k]) continue;
      const int j = x - R + q + k * RL;
      // OR only the bits not covered before this step (covered bits are
      // cleared only by a reset), so re-sensed rows cost no atomic
      const uint32_t ncov = rge[k] & ~rcov[k];
      or_field(cov + (size_t)j * RW, RW, c0, ncov);
      or_field(obst + (size_t)j * RW, RW, c0, rneg[k]);
      uint8_t* row_o = pl_obst + (size_t)j * L + c0;
      uint8_t* row_f = pl_free + (size_t)j * L + c0;
      // a cell covered before this step already holds 0 in _free: only new
      // cells (0 in _free) and obstacles (1 in layer P) are stored; fixed row
      // bases, so each store's column rides in its offset field
#pragma unroll
      for (int b = 0; b < n; ++b) {
        if ((rneg[k] >> b) & 1u) row_o[b] = 1;
        if ((ncov >> b) & 1u) row_f[b] = 0;
      }
    }
    const bool lead = me && q == 0;
    // robot cells: clear the old one, set the new one (use_scanning: a cell
    // vacated by one robot and entered by another keeps its 1)
    const bool moved = lead && (x != x_old || y != y_old);
    const size_t lay = (size_t)(s.scan ? 0 : i) * WL;
    bool reoccupied = false;
    if (s.scan && lead)
      for (int m = 0; m < N; ++m) reoccupied |= s_x[slot_env][m] == x_old && s_y[slot_env][m] == y_old;
    if (moved && !reoccupied) pl[lay + (size_t)x_old * L + y_old] = 0;
    if (moved) pl[lay + (size_t)x * L + y] = 1;
    // motion_penalty(a) on every slot (:203-208, 227-243)
    if ((qt < 0 || qt >= 4) && valid && li == 0) atomicOr(s.err, ERR_KEY);
    v = v + ((qt == ap) ? 0.0 : -1.0);
    if (lead) {
      if (!dpp) s_v[slot_env][slot] = v;
      s.pos[((size_t)e * N + i) * 2] = x;
      s.pos[((size_t)e * N + i) * 2 + 1] = y;
    }
    double total = 0.0;
    if (NG == 16 && dpp) {
      cnt = row_sum_to_lane0(cnt);  // group sum in lane 0
      // the slots' rewards from their quads, summed as np.sum does below 8
      // values: sequentially from -0.0 (np_pairwise_sum)
      const double v0 = row_share_f64<0>(v), v1 = row_share_f64<4>(v);
      const double v2 = row_share_f64<8>(v), v3 = row_share_f64<12>(v);
      total = -0.0;
      total += v0;
      if (N > 1) total += v1;
      if (N > 2) total += v2;
      if (N > 3) total += v3;
    } else {
#pragma unroll
      for (int o = NG / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);  // group sum
      wave_sync();
      if (valid && li == 0) total = np_pairwise_sum(s_v[slot_env], N);
    }
    if (valid && li == 0) {
      const int cs = cs0 + 1;
      const uint32_t cc = cc0 + (uint32_t)cnt;
      const double pc = (double)cc / (double)npos;
      const bool cond = (dt < 1.0 ? dt : 1.0) <= pc;  // min(_done_thresh, 1) <= percent_covered()
      if (cond) total = total + s.term;
      if (cond) s.done_thresh[e] = dt + s.dincr;  // done() (:408-411)
      dn = cond || (s.maxsteps > 0 && cs == s.maxsteps);
      s.a_prev[e] = qt;
      s.currstep[e] = cs;
      s.cov_cnt[e] = cc;
      reward[e] = total;
      done[e] = (uint8_t)dn;
      if (dn) {  // the episode record (Utils/utils.py:138-141)
        s.ep_pc[e] = pc;
        s.ep_len[e] = cs;
      }
    }
  }
  uint64_t rs = __ballot(s.auto_reset && valid && li == 0 && dn != 0);
  if (rs) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the step's map ORs land first
    const int e0 = blockIdx.x * (kEnvsPerBlock * GPW) + (int)(threadIdx.x >> 6) * GPW;
    for (; rs; rs &= rs - 1) {
      const int gj = (__ffsll((unsigned long long)rs) - 1) / NG;
      sg_reset_env(s, e0 + gj, lane, nullptr);
    }
  }
}

// --------------------------------------------------------------------------
// get_state (:305-317) planes: full rewrite of the uint8 layers (after a
// reset / state upload) and the distance layer of every env.
// --------------------------------------------------------------------------
// full rewrite of env e's uint8 layers (after a reset / state upload); the
// caller reads s.full[e] first (uniform) and this clears it
__device__ void write_full_layers(const SState& s, int e, int tid, int NT, int* s_px, int* s_py) {
  const int W = s.W, L = s.L, RW = s.RW, N = s.N;
  const size_t mw = (size_t)W * RW, WL = (size_t)W * L;
  const uint64_t* cov = s.cov + (size_t)e * mw;
  if (tid < N) {
    s_px[tid] = s.pos[((size_t)e * N + tid) * 2];
    s_py[tid] = s.pos[((size_t)e * N + tid) * 2 + 1];
  }
  uint8_t* pl = s.planes + (size_t)e * (s.P + 2) * WL;
  const uint64_t* ob = s.obst + (size_t)e * mw;
  for (size_t i = tid; i < WL; i += NT) {
    const int u = div_L(s, (int)i), v = (int)i - u * L;
    const size_t wi = (size_t)u * RW + (v >> 6);
    const int b = v & 63;
    for (int p = 0; p < s.P; ++p) pl[(size_t)p * WL + i] = 0;
    pl[(size_t)s.P * WL + i] = (uint8_t)((ob[wi] >> b) & 1ull);
    pl[(size_t)(s.P + 1) * WL + i] = (uint8_t)(((cov[wi] >> b) & 1ull) ^ 1ull);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < N) pl[(size_t)(s.scan ? 0 : tid) * WL + (size_t)s_px[tid] * L + s_py[tid]] = 1;
  if (tid == 0) s.full[e] = 0;
}

// LDS bytes of sg_erode_kernel: two bitboards, per-cell d (u8), the value LUT
__host__ __device__ inline size_t erode_lds_bytes(int W, int L) {
  const size_t nw = (size_t)W * ((L + 63) / 64);
  return 2 * nw * 8 + (((size_t)W * L + 15) & ~(size_t)15) + (((size_t)(W + L + 1) * 4 + 15) & ~(size_t)15);
}

// Distance layer by bit-parallel erosion (maps with W + L <= 257 whose
// planes fit LDS; every BASELINE-sized map).  With C = the sensed cells and
// cells outside the grid counting as non-sources (OpenCV's border), the L1
// distance to the nearest source is d(c) = #{k >= 0 : c in E_k}, E_0 = C,
// E_{k+1} = E_k & (its four 1-cell shifts): an L1 ball of radius k+1 is the
// radius-k ball grown by one 4-neighbour step.  A cell leaving at step k has
// d = k + 1; max(d) = the number of non-empty layers.  Each step is a few
// word ops per 64 cells, and max(d) is small (obstacles are sources), so the
// kernel is bound by the float32 layer write: per 4 cells one u32 of d from
// LDS, four LUT reads (1 - d/M, the reference's float32 steps), one 16-B store.
__global__ __launch_bounds__(256) void sg_erode_kernel(SState s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_px[kMaxAgents], s_py[kMaxAgents];
  const int e = blockIdx.x, tid = threadIdx.x, NT = blockDim.x;
  const int W = s.W, L = s.L, RW = s.RW;
  const int nw = W * RW;
  const size_t WL = (size_t)W * L;
  const bool was_full = s.full[e] != 0;  // read by every thread before it is cleared
  const int M_old = s.dist_M[e];
  if (tid < s.N) {  // robot cells (the region writes below), loaded while the map loads
    s_px[tid] = s.pos[((size_t)e * s.N + tid) * 2];
    s_py[tid] = s.pos[((size_t)e * s.N + tid) * 2 + 1];
  }
  if (was_full) write_full_layers(s, e, tid, NT, s_px, s_py);
  uint64_t* cur = reinterpret_cast<uint64_t*>(smem);
  uint64_t* nxt = cur + nw;
  uint8_t* d8 = reinterpret_cast<uint8_t*>(nxt + nw);
  float* lut = reinterpret_cast<float*>(d8 + ((WL + 15) & ~(size_t)15));
  const uint64_t* cov = s.cov + (size_t)e * nw;
  const uint64_t inval_last = (L & 63) ? ~low_mask(L & 63) : 0ull;  // bits >= L of a row's last word
  for (size_t i = tid; i < (WL + 15) / 16; i += NT) reinterpret_cast<uint4*>(d8)[i] = make_uint4(0, 0, 0, 0);
  int any_src = 0, any_cov = 0;
  for (int i = tid; i < nw; i += NT) {
    const int w = i % RW;
    const uint64_t inval = (w == RW - 1) ? inval_last : 0ull;
    const uint64_t c = cov[i] & ~inval;
    cur[i] = c | inval;
    any_src |= (~c & ~inval) != 0ull;
    any_cov |= c != 0ull;
  }
  any_src = __syncthreads_or(any_src);
  any_cov = __syncthreads_or(any_cov);
  float* out = s.dist_plane + (size_t)e * WL;
  if (!any_src) {  // no source cell: SciPy's -1 everywhere -> 1 - (-1)
    for (size_t i = tid; i < WL; i += NT) out[i] = 2.0f;
    if (tid == 0) s.dist_M[e] = -2;
    return;
  }
  int M = 0;
  if (any_cov) {
    // word i = u * RW + w: divided once per thread, then advanced by NT with a carry
    const int u0 = tid / RW, w0 = tid - u0 * RW;
    const int st_u = NT / RW, st_w = NT - st_u * RW;
    for (int k = 0;; ++k) {
      int nz = 0;
      int u = u0, w = w0;
      for (int i = tid; i < nw; i += NT) {
        const uint64_t inval = (w == RW - 1) ? inval_last : 0ull;
        const uint64_t c = cur[i];
        const uint64_t up = u > 0 ? cur[i - RW] : ~0ull;
        const uint64_t dn = u < W - 1 ? cur[i + RW] : ~0ull;
        const uint64_t lw = w > 0 ? cur[i - 1] : ~0ull;
        const uint64_t rw = w < RW - 1 ? cur[i + 1] : ~0ull;
        const uint64_t n = (c & up & dn & ((c << 1) | (lw >> 63)) & ((c >> 1) | (rw << 63))) | inval;
        nxt[i] = n;
        uint64_t leave = c & ~n;
        if (leave) {
          uint8_t* row = d8 + (size_t)u * L + (w << 6);
          const uint8_t dk = (uint8_t)(k + 1);
          for (; leave; leave &= leave - 1) row[__ffsll((unsigned long long)leave) - 1] = dk;
        }
        nz |= (n & ~inval) != 0ull;
        w += st_w;
        const int cw = w >= RW;
        w -= cw ? RW : 0;
        u += st_u + cw;
      }
      if (!__syncthreads_or(nz)) {
        M = k + 1;
        break;
      }
      uint64_t* t = cur;
      cur = nxt;
      nxt = t;
    }
  }
  const float Mf = (float)M;
  for (int d = tid; d <= M; d += NT) lut[d] = dist_value((float)d, Mf);
  if (tid == 0) s.dist_M[e] = M;
  // Since the layer was last written only this step's sensing changed the
  // map: newly covered cells n lie in the robots' windows (|n - p_i| <= r,
  // Chebyshev), and a cell's d changes only if its nearest source was such a
  // cell, i.e. |c - n|_1 <= d_old(c) <= M_old.  So with max(d) unchanged every
  // changed value lies within r + M_old of a robot, and the rest of the layer
  // already holds the exact new values.  A changed max, a full-rewrite flag
  // (reset / state upload) or MARLCOV_SG_FULL_DIST rewrites the whole layer.
  const int h = s.r + (M_old > 0 ? M_old : 0) + 1, side = 2 * h + 1;
  const bool all = was_full || s.dist_full || M != M_old || M_old < 0 ||
                   (size_t)s.N * side * side >= WL;
  __syncthreads();
  if (!all) {
    // idx = (i * side + rr) * side + cc, divided once and then advanced by NT
    // with carries (each digit step is < side, so one subtraction each)
    const int per = side * side;
    const int q_nt = NT / side, st_cc = NT - q_nt * side;
    const int st_i = q_nt / side, st_rr = q_nt - st_i * side;
    int i = tid / per;
    int rr = (tid - i * per) / side;
    int cc = tid - i * per - rr * side;
    for (int idx = tid; idx < s.N * per; idx += NT) {
      const int u = s_px[i] - h + rr;
      const int v = s_py[i] - h + cc;
      if (u >= 0 && u < W && v >= 0 && v < L) out[(size_t)u * L + v] = lut[d8[(size_t)u * L + v]];
      cc += st_cc;
      int c = cc >= side;
      cc -= c ? side : 0;
      rr += st_rr + c;
      c = rr >= side;
      rr -= c ? side : 0;
      i += st_i + c;
    }
  } else if ((L & 3) == 0) {
    const uint32_t* d4 = reinterpret_cast<const uint32_t*>(d8);
    float4* o4 = reinterpret_cast<float4*>(out);
    for (size_t g = tid; g < WL / 4; g += NT) {
      const uint32_t q = d4[g];
      o4[g] = make_float4(lut[q & 255u], lut[(q >> 8) & 255u], lut[(q >> 16) & 255u], lut[q >> 24]);
    }
  } else {
    for (size_t i = tid; i < WL; i += NT) out[i] = lut[d8[i]];
  }
}

// Distance layer by separable sweeps (any map up to kMaxSide): a row pass
// (distance along the row) and down/up min-plus column sweeps over u16
// planes in LDS or, when they do not fit, the global scratch.
template <bool kLds>
__global__ __launch_bounds__(256) void sg_dist_kernel(SState s, int pitch) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_px[kMaxAgents], s_py[kMaxAgents];
  __shared__ int s_max;
  const int e = blockIdx.x, tid = threadIdx.x, NT = blockDim.x;
  const int W = s.W, L = s.L, RW = s.RW;
  const size_t mw = (size_t)W * RW, WL = (size_t)W * L;
  const uint64_t* cov = s.cov + (size_t)e * mw;
  uint16_t* H = kLds ? reinterpret_cast<uint16_t*>(smem) : s.scratch + (size_t)e * W * pitch;
  if (tid == 0) s_max = 0;
  if (s.full[e]) write_full_layers(s, e, tid, NT, s_px, s_py);

  // row pass: H[u][v] = distance along row u to the nearest source (_free != 0)
  for (int u = tid; u < W; u += NT) {
    const uint64_t* row = cov + (size_t)u * RW;
    uint16_t* h = H + (size_t)u * pitch;
    int last = -(1 << 20);
    for (int wv = 0; wv < RW; ++wv) {
      const int nb = min(64, L - wv * 64);
      const uint64_t src = ~row[wv] & low_mask(nb);
      if (src == low_mask(nb)) {  // no sensed cell in this word
        for (int b = 0; b < nb; ++b) h[wv * 64 + b] = 0;
        last = wv * 64 + nb - 1;
        continue;
      }
      for (int b = 0; b < nb; ++b) {
        const int v = wv * 64 + b;
        if ((src >> b) & 1ull) last = v;
        h[v] = (uint16_t)min(v - last, kInfD);
      }
    }
    int next = 1 << 21;
    for (int wv = RW - 1; wv >= 0; --wv) {
      const int nb = min(64, L - wv * 64);
      const uint64_t src = ~row[wv] & low_mask(nb);
      if (src == low_mask(nb)) {
        next = wv * 64;
        continue;
      }
      for (int b = nb - 1; b >= 0; --b) {
        const int v = wv * 64 + b;
        if ((src >> b) & 1ull) next = v;
        const int hv = h[v];
        if (next - v < hv) h[v] = (uint16_t)(next - v);
      }
    }
  }
  __syncthreads();
  // column pass: d(u, v) = min_u' |u - u'| + H[u'][v], down then up
  int mx = 0;
  for (int v = tid; v < L; v += NT) {
    int f = 1 << 20;
    for (int u = 0; u < W; ++u) {
      f = min(f + 1, (int)H[(size_t)u * pitch + v]);
      H[(size_t)u * pitch + v] = (uint16_t)min(f, kInfD);
    }
    f = 1 << 20;
    for (int u = W - 1; u >= 0; --u) {
      f = min(f + 1, (int)H[(size_t)u * pitch + v]);
      H[(size_t)u * pitch + v] = (uint16_t)min(f, kInfD);
      mx = max(mx, min(f, kInfD));
    }
  }
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  if ((tid & 63) == 0) atomicMax(&s_max, mx);
  __syncthreads();
  const int M = s_max;
  float* out = s.dist_plane + (size_t)e * WL;
  if (M >= kInfD) {  // no source cell: SciPy's -1 everywhere -> 1 - (-1)
    for (size_t i = tid; i < WL; i += NT) out[i] = 2.0f;
    return;
  }
  const float Mf = (float)M;
  for (size_t i = tid; i < WL; i += NT) {
    const int u = div_L(s, (int)i), v = (int)i - u * L;
    out[i] = dist_value((float)H[(size_t)u * pitch + v], Mf);
  }
}

// --------------------------------------------------------------------------
// grid pool: int8 [G][W][L] -> bit rows, numpos; Bernoulli generation
// --------------------------------------------------------------------------
__global__ void sg_pack_kernel(SState s, const int8_t* __restrict__ grids, uint64_t* gneg,
                               uint64_t* gpos, int32_t* numpos) {
  const size_t total = (size_t)s.G * s.W * s.RW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int wv = (int)(i % s.RW);
    const size_t gx = i / s.RW;
    const int x = (int)(gx % s.W), g = (int)(gx / s.W);
    const int8_t* src = grids + ((size_t)g * s.W + x) * s.L;
    uint64_t neg = 0, pos = 0;
    for (int b = 0; b < 64 && wv * 64 + b < s.L; ++b) {
      const int8_t c = src[wv * 64 + b];
      neg |= (uint64_t)(c < 0) << b;
      pos |= (uint64_t)(c > 0) << b;
    }
    gneg[i] = neg;
    gpos[i] = pos;
    if (pos) atomicAdd(&numpos[g], __popcll(pos));
  }
}

__global__ void sg_gen_kernel(SState s, uint64_t seed, uint32_t thresh, uint64_t* gneg, uint64_t* gpos,
                              int32_t* numpos) {
  const size_t total = (size_t)s.G * s.W * s.RW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int wv = (int)(i % s.RW);
    const size_t gx = i / s.RW;
    const int x = (int)(gx % s.W), g = (int)(gx / s.W);
    const int nb = min(64, s.L - wv * 64);
    uint64_t neg = 0;
    for (int q = 0; q < 16; ++q) {
      const uint4 r = philox(seed, make_uint4((uint32_t)x, (uint32_t)wv, s.grid0 + (uint32_t)g, 0x5367656eu + ((uint32_t)q << 28)));
      neg |= (uint64_t)(r.x < thresh) << (4 * q);
      neg |= (uint64_t)(r.y < thresh) << (4 * q + 1);
      neg |= (uint64_t)(r.z < thresh) << (4 * q + 2);
      neg |= (uint64_t)(r.w < thresh) << (4 * q + 3);
    }
    neg &= low_mask(nb);
    const uint64_t pos = ~neg & low_mask(nb);
    gneg[i] = neg;
    gpos[i] = pos;
    if (pos) atomicAdd(&numpos[g], __popcll(pos));
  }
}

}  // namespace mcs

// ==========================================================================
// C ABI
// ==========================================================================
namespace {

int sg_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int sg_fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  mc::set_last_error(buf);
  return code;
}

#define SG_TRY(expr)                                                                       \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) return sg_fail(MC_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

struct SgEnv {
  mc_sg_config cfg;
  mcs::SState s;
  mc_sg_layout lay;
  int device = 0;
  int pitch = 0;      // u16 elements per distance-plane row
  bool lds = true;    // distance planes in LDS (else s.scratch)
  bool erode = false; // sg_erode_kernel (else the sweep kernel)
  size_t erode_lds = 0;
  int dist_nt = 256;
  bool grids_set = false;
  bool stale = true;  // the dist layer does not describe the current maps
  bool rows = true;   // row-parallel step kernel when it applies (MARLCOV_SG_ROWS)
  std::vector<void*> allocs;
};

SgEnv* as_sg(void* p) { return static_cast<SgEnv*>(p); }

int sg_alloc(SgEnv* E, void** p, size_t bytes) {
  void* q = nullptr;
  SG_TRY(hipMalloc(&q, bytes < 16 ? 16 : bytes));
  SG_TRY(hipMemset(q, 0, bytes < 16 ? 16 : bytes));
  E->allocs.push_back(q);
  E->lay.state_bytes += (int64_t)bytes;
  *p = q;
  return MC_OK;
}

struct SgField {
  void* ptr;
  int64_t bytes;
};

SgField sg_field(SgEnv* E, int f) {
  const mcs::SState& s = E->s;
  const int64_t B = s.B, N = s.N, G = s.G, mw = (int64_t)s.W * s.RW;
  switch (f) {
    case MC_SG_FIELD_POS: return {s.pos, B * N * 8};
    case MC_SG_FIELD_COVERED: return {s.cov, B * mw * 8};
    case MC_SG_FIELD_OBST: return {s.obst, B * mw * 8};
    case MC_SG_FIELD_COV_COUNT: return {s.cov_cnt, B * 4};
    case MC_SG_FIELD_CURRSTEP: return {s.currstep, B * 4};
    case MC_SG_FIELD_DONE_THRESH: return {s.done_thresh, B * 8};
    case MC_SG_FIELD_A_PREV: return {s.a_prev, B * 4};
    case MC_SG_FIELD_ENV_GRID: return {s.env_grid, B * 4};
    case MC_SG_FIELD_EPISODE: return {s.episode, B * 4};
    case MC_SG_FIELD_NUMPOS: return {(void*)s.numpos, G * 4};
    case MC_SG_FIELD_GRID_NEG: return {(void*)s.gneg, G * mw * 8};
    case MC_SG_FIELD_GRID_POS: return {(void*)s.gpos, G * mw * 8};
    case MC_SG_FIELD_EP_PC: return {s.ep_pc, B * 8};
    case MC_SG_FIELD_EP_LEN: return {s.ep_len, B * 4};
    default: return {nullptr, -1};
  }
}

int sg_ready(SgEnv* E, const char* who) {
  if (!E->grids_set) return sg_fail(MC_ESTATE, "%s: grids not set (mc_sg_set_grids / mc_sg_generate_grids)", who);
  if (!E->s.planes || !E->s.dist_plane) return sg_fail(MC_ESTATE, "%s: state buffers not registered (mc_sg_set_obs)", who);
  return MC_OK;
}

hipError_t launch_dist(SgEnv* E, hipStream_t st) {
  if (E->erode) {
    hipLaunchKernelGGL(mcs::sg_erode_kernel, dim3(E->s.B), dim3(256), E->erode_lds, st, E->s);
    return hipGetLastError();
  }
  const size_t lds = E->lds ? (size_t)E->s.W * E->pitch * 2 : 0;
  if (E->lds)
    hipLaunchKernelGGL(mcs::sg_dist_kernel<true>, dim3(E->s.B), dim3(E->dist_nt), lds, st, E->s, E->pitch);
  else
    hipLaunchKernelGGL(mcs::sg_dist_kernel<false>, dim3(E->s.B), dim3(E->dist_nt), 0, st, E->s, E->pitch);
  return hipGetLastError();
}

int check_numpos(SgEnv* E, hipStream_t st) {
  std::vector<int32_t> np(E->s.G);
  SG_TRY(hipMemcpyAsync(np.data(), E->s.numpos, np.size() * 4, hipMemcpyDeviceToHost, st));
  SG_TRY(hipStreamSynchronize(st));
  for (int g = 0; g < E->s.G; ++g)
    if (np[g] <= 0)
      return sg_fail(MC_EINVAL,
                     "grid %d has no cell > 0: percent_covered() divides by count_nonzero(grid > 0) "
                     "(super_grid_rl.py:420-421)",
                     g);
  E->grids_set = true;
  return MC_OK;
}

}  // namespace

extern "C" {

int mc_sg_create(const mc_sg_config* cfg, int hip_device, void** out_env) {
  if (!cfg || !out_env) return sg_fail(MC_EINVAL, "mc_sg_create: null argument");
  const mc_sg_config& c = *cfg;
  if (c.num_envs < 1) return sg_fail(MC_EINVAL, "num_envs must be >= 1");
  if (c.num_agents < 1 || c.num_agents > mcs::kMaxAgents) return sg_fail(MC_EINVAL, "numrobot must be in [1, 64]");
  if (c.width < 1 || c.length < 1 || c.width > mcs::kMaxSide || c.length > mcs::kMaxSide)
    return sg_fail(MC_EINVAL, "grid sides must be in [1, %d]", mcs::kMaxSide);
  if ((int64_t)c.width * c.length < c.num_agents) return sg_fail(MC_EINVAL, "more robots than cells");
  if (c.num_grids < 1) return sg_fail(MC_EINVAL, "num_grids must be >= 1");
  if (c.senseradius < 0 || c.senseradius > mcs::kMaxRadius) return sg_fail(MC_EINVAL, "senseradius must be in [0, 15]");
  SG_TRY(hipSetDevice(hip_device));
  SgEnv* E = new SgEnv();
  E->cfg = c;
  E->device = hip_device;
  E->lay = mc_sg_layout{};
  mcs::SState& s = E->s;
  s = mcs::SState{};
  s.B = c.num_envs;
  s.N = c.num_agents;
  s.W = c.width;
  s.L = c.length;
  s.G = c.num_grids;
  s.RW = (c.length + 63) / 64;
  s.r = c.senseradius;
  s.P = c.use_scanning ? 1 : c.num_agents;
  s.pen = c.collision_penalty;
  s.fpen = c.free_penalty;
  s.term = c.terminal_reward;
  s.dincr = c.done_incr;
  s.dist = c.dist_reward != 0;
  s.scan = c.use_scanning != 0;
  s.maxsteps = c.maxsteps;
  s.auto_reset = c.auto_reset != 0;
  s.grid_mode = c.reset_grid_mode;
  s.mg_L = mc::magic_div((uint32_t)c.length);
  {
    const char* fd = getenv("MARLCOV_SG_FULL_DIST");
    s.dist_full = fd && atoi(fd) == 1;
    // MARLCOV_SG_ROWS=0: one lane per robot instead of the row-parallel step
    // kernel (read per handle: the parity suite runs both)
    const char* rw = getenv("MARLCOV_SG_ROWS");
    E->rows = !(rw && atoi(rw) == 0);
  }
  s.seed = c.seed;
  s.env0 = c.env_offset;
  s.grid0 = c.grid_offset;
  // distance planes: u16 rows with an odd dword pitch (the row pass writes
  // column v of W rows at once: distinct banks)
  E->pitch = ((c.length + 1) / 2) * 2;
  if (((E->pitch / 2) & 1) == 0) E->pitch += 2;
  E->lds = (size_t)c.width * E->pitch * 2 <= mcs::kLdsLimit;
  E->erode_lds = mcs::erode_lds_bytes(c.width, c.length);
  static const bool force_sweep = [] {  // MARLCOV_SG_SWEEP=1: A/B against the sweep kernel
    const char* v = getenv("MARLCOV_SG_SWEEP");
    return v && atoi(v) == 1;
  }();
  E->erode = !force_sweep && c.width + c.length <= 257 && E->erode_lds <= mcs::kLdsLimit;
  const int side = c.width > c.length ? c.width : c.length;
  E->dist_nt = side <= 64 ? 64 : (side <= 128 ? 128 : 256);
  const size_t B = s.B, N = s.N, G = s.G, mw = (size_t)s.W * s.RW;
  void* p;
  int rc = 0;
#define SG_ALLOC(field, type, bytes)        \
  rc = sg_alloc(E, &p, (bytes));            \
  if (rc) { mc_sg_destroy(E); return rc; }  \
  s.field = (type)p;
  SG_ALLOC(gneg, const uint64_t*, G * mw * 8);
  SG_ALLOC(gpos, const uint64_t*, G * mw * 8);
  SG_ALLOC(numpos, const int32_t*, G * 4);
  SG_ALLOC(env_grid, int32_t*, B * 4);
  SG_ALLOC(pos, int32_t*, B * N * 8);
  SG_ALLOC(cov, uint64_t*, B * mw * 8);
  SG_ALLOC(obst, uint64_t*, B * mw * 8);
  SG_ALLOC(cov_cnt, uint32_t*, B * 4);
  SG_ALLOC(currstep, int32_t*, B * 4);
  SG_ALLOC(done_thresh, double*, B * 8);
  SG_ALLOC(a_prev, int32_t*, B * 4);
  SG_ALLOC(episode, uint32_t*, B * 4);
  SG_ALLOC(full, uint8_t*, B);
  SG_ALLOC(dist_M, int32_t*, B * 4);
  SG_ALLOC(ep_pc, double*, B * 8);
  SG_ALLOC(ep_len, int32_t*, B * 4);
  SG_ALLOC(err, uint32_t*, 4);
  if (!E->lds) {
    SG_ALLOC(scratch, uint16_t*, B * s.W * E->pitch * 2);
  }
#undef SG_ALLOC
  {
    std::vector<int32_t> eg(B), ap(B, -1);
    std::vector<double> dt(B, c.done_thresh);
    std::vector<uint8_t> fl(B, 1);
    for (size_t e = 0; e < B; ++e) eg[e] = (int32_t)(e % G);
    hipError_t he = hipMemcpy(s.env_grid, eg.data(), B * 4, hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(s.a_prev, ap.data(), B * 4, hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(s.done_thresh, dt.data(), B * 8, hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(s.full, fl.data(), B, hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemset(s.dist_M, 0xFF, B * 4);
    if (he != hipSuccess) {
      mc_sg_destroy(E);
      return sg_fail(MC_EHIP, "mc_sg_create: %s", hipGetErrorString(he));
    }
  }
  E->lay.pos_layers = s.P;
  E->lay.obs_layers = s.P + 2;
  E->lay.row_words = s.RW;
  *out_env = E;
  return MC_OK;
}

void mc_sg_destroy(void* env) {
  SgEnv* E = as_sg(env);
  if (!E) return;
  (void)hipSetDevice(E->device);
  for (void* p : E->allocs) (void)hipFree(p);
  delete E;
}

int mc_sg_query(void* env, mc_sg_layout* out) {
  SgEnv* E = as_sg(env);
  if (!E || !out) return sg_fail(MC_EINVAL, "mc_sg_query: null argument");
  *out = E->lay;
  return MC_OK;
}

int mc_sg_set_grids(void* env, const int8_t* dev_grids, int32_t num_grids, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E || !dev_grids) return sg_fail(MC_EINVAL, "mc_sg_set_grids: null argument");
  if (num_grids != E->s.G) return sg_fail(MC_EINVAL, "mc_sg_set_grids: %d grids, config says %d", num_grids, E->s.G);
  hipStream_t st = (hipStream_t)stream;
  SG_TRY(hipSetDevice(E->device));
  SG_TRY(hipMemsetAsync((void*)E->s.numpos, 0, (size_t)E->s.G * 4, st));
  const size_t total = (size_t)E->s.G * E->s.W * E->s.RW;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  hipLaunchKernelGGL(mcs::sg_pack_kernel, dim3(blocks), dim3(256), 0, st, E->s, dev_grids,
                     (uint64_t*)E->s.gneg, (uint64_t*)E->s.gpos, (int32_t*)E->s.numpos);
  SG_TRY(hipGetLastError());
  SG_TRY(hipMemsetAsync(E->s.full, 1, (size_t)E->s.B, st));  // new obstacles: every layer value may change
  E->stale = true;
  return check_numpos(E, st);
}

int mc_sg_generate_grids(void* env, uint64_t seed, double p_obst, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E) return sg_fail(MC_EINVAL, "mc_sg_generate_grids: null env");
  if (!(p_obst >= 0.0 && p_obst < 1.0)) return sg_fail(MC_EINVAL, "p_obst must be in [0, 1)");
  hipStream_t st = (hipStream_t)stream;
  SG_TRY(hipSetDevice(E->device));
  SG_TRY(hipMemsetAsync((void*)E->s.numpos, 0, (size_t)E->s.G * 4, st));
  const size_t total = (size_t)E->s.G * E->s.W * E->s.RW;
  const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  const uint32_t thresh = (uint32_t)(p_obst * 4294967296.0);
  hipLaunchKernelGGL(mcs::sg_gen_kernel, dim3(blocks), dim3(256), 0, st, E->s, seed, thresh,
                     (uint64_t*)E->s.gneg, (uint64_t*)E->s.gpos, (int32_t*)E->s.numpos);
  SG_TRY(hipGetLastError());
  SG_TRY(hipMemsetAsync(E->s.full, 1, (size_t)E->s.B, st));  // new obstacles: every layer value may change
  E->stale = true;
  return check_numpos(E, st);
}

int mc_sg_set_env_grids(void* env, const int32_t* dev_env_grid, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E || !dev_env_grid) return sg_fail(MC_EINVAL, "mc_sg_set_env_grids: null argument");
  SG_TRY(hipSetDevice(E->device));
  SG_TRY(hipMemcpyAsync(E->s.env_grid, dev_env_grid, (size_t)E->s.B * 4, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream));
  SG_TRY(hipMemsetAsync(E->s.full, 1, (size_t)E->s.B, (hipStream_t)stream));
  E->stale = true;
  return MC_OK;
}

int mc_sg_set_obs(void* env, uint8_t* dev_planes, float* dev_dist) {
  SgEnv* E = as_sg(env);
  if (!E || !dev_planes || !dev_dist) return sg_fail(MC_EINVAL, "mc_sg_set_obs: null argument");
  E->s.planes = dev_planes;
  E->s.dist_plane = dev_dist;
  SG_TRY(hipSetDevice(E->device));
  SG_TRY(hipMemset(E->s.full, 1, (size_t)E->s.B));
  E->stale = true;
  return MC_OK;
}

int mc_sg_reset(void* env, const uint8_t* dev_env_mask, const int32_t* dev_pos, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E) return sg_fail(MC_EINVAL, "mc_sg_reset: null env");
  int rc = sg_ready(E, "mc_sg_reset");
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  SG_TRY(hipSetDevice(E->device));
  const int blocks = (E->s.B + mcs::kEnvsPerBlock - 1) / mcs::kEnvsPerBlock;
  hipLaunchKernelGGL(mcs::sg_reset_kernel, dim3(blocks), dim3(64 * mcs::kEnvsPerBlock), 0, st, E->s,
                     dev_env_mask, dev_pos);
  SG_TRY(hipGetLastError());
  SG_TRY(launch_dist(E, st));
  E->stale = false;
  return MC_OK;
}

int mc_sg_step(void* env, const uint8_t* dev_actions, const int32_t* dev_quot, double* dev_reward,
               uint8_t* dev_done, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E || !dev_actions || !dev_reward || !dev_done) return sg_fail(MC_EINVAL, "mc_sg_step: null argument");
  int rc = sg_ready(E, "mc_sg_step");
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  SG_TRY(hipSetDevice(E->device));
  if (E->stale) SG_TRY(launch_dist(E, st));  // the pre-move distance_map of the current maps
  // envs per wave: as many groups of (N rounded up to a power of two) lanes
  // as fit 64, capped at 4 (MARLCOV_SG_GPW overrides the cap).  sg_c2
  // (tools/gpu_sg_gpw.sh, rocprof): 1 17.8 us, 2 14.3, 4 12.8, 8 14.6, 16 19.4
  // -- past 4 envs per wave there are too few waves to hide the window loads
  static const int gpw_cap = [] {
    const char* v = getenv("MARLCOV_SG_GPW");
    const int c = v ? atoi(v) : 4;
    return c >= 1 ? c : 4;
  }();
  int gpw = 1;
  while (gpw < 16 && 2 * gpw <= gpw_cap && E->s.N <= 64 / (2 * gpw)) gpw *= 2;
  static const bool force_generic = [] {  // MARLCOV_SG_GENERIC=1: A/B against the runtime-radius kernel
    const char* v = getenv("MARLCOV_SG_GENERIC");
    return v && atoi(v) == 1;
  }();
  const int R = force_generic ? -1 : (E->s.r >= 1 && E->s.r <= 3 ? E->s.r : -1);
  decltype(&mcs::sg_step_kernel<-1, 1>) kern = nullptr;
  // compiled radius and at least 4 lanes per robot: the row-parallel kernel
  // (MARLCOV_SG_ROWS=0 at create keeps one lane per robot)
  int p2 = 1;
  while (p2 < E->s.N) p2 *= 2;
  if (E->rows && R >= 1 && 4 * p2 <= 64) {
    gpw = 1;
    while (2 * gpw <= gpw_cap && 4 * p2 * 2 * gpw <= 64) gpw *= 2;
#define SG_PICK_ROWS(RR)                                             \
  switch (gpw) {                                                     \
    case 1: kern = mcs::sg_step_rows<RR, 1>; break;                  \
    case 2: kern = mcs::sg_step_rows<RR, 2>; break;                  \
    case 4: kern = mcs::sg_step_rows<RR, 4>; break;                  \
    default: kern = mcs::sg_step_rows<RR, 8>; break;                 \
  }
    switch (R) {
      case 1: SG_PICK_ROWS(1); break;
      case 2: SG_PICK_ROWS(2); break;
      default: SG_PICK_ROWS(3); break;
    }
#undef SG_PICK_ROWS
  }
#define SG_PICK(RR)                                                  \
  switch (gpw) {                                                     \
    case 1: kern = mcs::sg_step_kernel<RR, 1>; break;                \
    case 2: kern = mcs::sg_step_kernel<RR, 2>; break;                \
    case 4: kern = mcs::sg_step_kernel<RR, 4>; break;                \
    case 8: kern = mcs::sg_step_kernel<RR, 8>; break;                \
    default: kern = mcs::sg_step_kernel<RR, 16>; break;              \
  }
  if (kern == nullptr) {
    switch (R) {  // compile-time radii of the reference configs (staged window)
      case 1: SG_PICK(1); break;
      case 2: SG_PICK(2); break;
      case 3: SG_PICK(3); break;
      default: SG_PICK(-1); break;
    }
  }
#undef SG_PICK
  const int per_block = mcs::kEnvsPerBlock * gpw;
  const int blocks = (E->s.B + per_block - 1) / per_block;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64 * mcs::kEnvsPerBlock), 0, st, E->s, dev_actions, dev_quot,
                     dev_reward, dev_done);
  SG_TRY(hipGetLastError());
  SG_TRY(launch_dist(E, st));
  E->stale = false;
  return MC_OK;
}

int64_t mc_sg_field_bytes(void* env, int32_t f) {
  SgEnv* E = as_sg(env);
  if (!E) return sg_fail(MC_EINVAL, "mc_sg_field_bytes: null env");
  SgField d = sg_field(E, f);
  if (!d.ptr) return sg_fail(MC_EINVAL, "unknown state field %d", f);
  return d.bytes;
}

int mc_sg_get_state(void* env, int32_t f, void* dev_dst, int64_t bytes, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E || !dev_dst) return sg_fail(MC_EINVAL, "mc_sg_get_state: null argument");
  SgField d = sg_field(E, f);
  if (!d.ptr) return sg_fail(MC_EINVAL, "unknown state field %d", f);
  if (bytes != d.bytes) return sg_fail(MC_EINVAL, "field %d is %lld bytes, got %lld", f, (long long)d.bytes, (long long)bytes);
  SG_TRY(hipSetDevice(E->device));
  SG_TRY(hipMemcpyAsync(dev_dst, d.ptr, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MC_OK;
}

int mc_sg_set_state(void* env, int32_t f, const void* dev_src, int64_t bytes, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E || !dev_src) return sg_fail(MC_EINVAL, "mc_sg_set_state: null argument");
  SgField d = sg_field(E, f);
  if (!d.ptr) return sg_fail(MC_EINVAL, "unknown state field %d", f);
  if (f == MC_SG_FIELD_EP_PC || f == MC_SG_FIELD_EP_LEN) return sg_fail(MC_EINVAL, "field %d is read-only", f);
  if (bytes != d.bytes) return sg_fail(MC_EINVAL, "field %d is %lld bytes, got %lld", f, (long long)d.bytes, (long long)bytes);
  hipStream_t st = (hipStream_t)stream;
  SG_TRY(hipSetDevice(E->device));
  SG_TRY(hipMemcpyAsync(d.ptr, dev_src, (size_t)bytes, hipMemcpyDeviceToDevice, st));
  if (f == MC_SG_FIELD_GRID_NEG || f == MC_SG_FIELD_GRID_POS || f == MC_SG_FIELD_NUMPOS) E->grids_set = true;
  SG_TRY(hipMemsetAsync(E->s.full, 1, (size_t)E->s.B, st));
  E->stale = true;
  return MC_OK;
}

int mc_sg_check(void* env, void* stream) {
  SgEnv* E = as_sg(env);
  if (!E) return sg_fail(MC_EINVAL, "mc_sg_check: null env");
  hipStream_t st = (hipStream_t)stream;
  SG_TRY(hipSetDevice(E->device));
  uint32_t err = 0;
  SG_TRY(hipMemcpyAsync(&err, E->s.err, 4, hipMemcpyDeviceToHost, st));
  SG_TRY(hipStreamSynchronize(st));
  if (err) {
    SG_TRY(hipMemsetAsync(E->s.err, 0, 4, st));
    SG_TRY(hipStreamSynchronize(st));
    return sg_fail(MC_EDEVICE, "device error word 0x%x (4=placement 8=inject 16=motion_penalty KeyError)", err);
  }
  return MC_OK;
}

}  // extern "C"
