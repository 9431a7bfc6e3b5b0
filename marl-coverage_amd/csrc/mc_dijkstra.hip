// mc_dijkstra.hip — the dijkstra_input observation layer.
//
// Reference: Environments/dijkstra.py:112-187 dijkstra_path_map, called from
// Environments/dec_grid_rl.py:354-358 as
//   dijkstra_path_map(free_pad[i] - obst_pad[i], x + pad, y + pad)
// and cropped E x E around the robot into obs layer 3.  On the map
// g = free - obst (1 explored, 0 unexplored, -1 obstacle; the pad ring is 0)
// a PriorityQueue of (cost, (x, y)) pops cells in BFS order, ties by (x, y);
// the first popped 0-cell is the end point; the path is then walked back from
// it, at each cell taking the first neighbour in the order +x, -x, +y, -y whose
// cost is one less.
//
// GPU form, two kernels.  The window kernel runs one wave per (env, agent)
// on the 64 x 64 cells (8 x 8 tiles) around the robot, one window row per
// lane in registers: a BFS layer is two cross-lane shifts and a few bit
// operations, no LDS and no barrier.  Every cell of BFS layer j lies within
// L1 distance j of the start, and the robot sits at least 24 cells inside
// the window on every side, so layers 1..24 (and the walk back, which stays
// on cells of cost < d*) are exact in the window; an (env, agent) whose
// nearest unexplored cell is farther is appended to a device list that the
// full kernel (below) then solves on the whole map.
//
// Full kernel: one workgroup per listed (env, agent).  The map is held in LDS
// as row bitboards (one bit per cell, 64 columns per word) over the
// pad-extended grid.  BFS layer j is dilate(layer j-1) & ~reached & ~obstacle: a whole
// layer per step of bit operations.  The pop order inside a layer only
// matters for the end point, which is the (x, y)-smallest 0-cell of the first
// layer that holds one — a workgroup min.  For the walk back only cost mod 3
// is kept (two bitboards): a neighbour of a cost-j cell has cost j-1, j or
// j+1, and mod 3 tells them apart.  Four lanes test the four neighbours of
// the walk in parallel; the first valid one in reference order wins.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "mc_bitboard.h"

namespace mc {

namespace {

constexpr int kDjThreads = 256;
constexpr unsigned kDjFullGrid = 256;  // workgroups of the full-map kernel over the listed items

struct DjLds {
  uint64_t *ob, *tg, *bl, *f0, *f1, *m0, *m1;
  uint64_t *tf, *to;  // the agent's free / obstacle tiles
};

}  // namespace

// one (env, agent) on the whole map; every thread of the workgroup calls it
__device__ __forceinline__ void dijkstra_full(const State& s, int pad, int layer, int Lc,
                                              uint8_t* __restrict__ obs_out, int e, int a,
                                              char* smem) {
  __shared__ int s_end[3], s_any[3];  // per BFS layer j: slot j % 3
  __shared__ uint32_t s_crop[32];
  const int tid = threadIdx.x;
  const int RX = s.Wp + 2 * pad, RY = s.Lp + 2 * pad, RW = (RY + 63) >> 6, NW = RX * RW;
  const int mt = s.MT;
  DjLds L;
  uint64_t* p = reinterpret_cast<uint64_t*>(smem);
  L.ob = p;
  L.tg = p + NW;
  L.bl = p + 2 * NW;
  L.f0 = p + 3 * NW;
  L.f1 = p + 4 * NW;
  L.m0 = p + 5 * NW;
  L.m1 = p + 6 * NW;
  L.tf = p + 7 * NW;
  L.to = L.tf + mt;

  // the agent's maps (tiles) and start cell
  const size_t fb = ((size_t)e * s.N + a) * mt;
  for (int i = tid; i < mt; i += kDjThreads) {
    L.tf[i] = s.freem[fb + i];
    L.to[i] = s.obstm[fb + i];
  }
  const int sx = s.pos[((size_t)e * s.N + a) * 2] + pad;
  const int sy = s.pos[((size_t)e * s.N + a) * 2 + 1] + pad;
  if (tid < 32) s_crop[tid] = 0;
  if (tid < 3) {
    s_end[tid] = INT32_MAX;
    s_any[tid] = 0;
  }
  __syncthreads();
  // g = free - obst: obstacle where only obst is set, target (0) where both or
  // neither are; columns past the extended grid are neither
  const uint64_t last = (RY & 63) ? low_mask(RY & 63) : ~0ull;
  for (int i = tid; i < NW; i += kDjThreads) {
    const int u = i / RW, w = i - u * RW;
    uint64_t f, o;
    f = row_word(s, L.tf, pad, u, w);
    o = row_word(s, L.to, pad, u, w);
    const uint64_t in = (w == RW - 1) ? last : ~0ull;
    L.ob[i] = o & ~f & in;
    L.tg[i] = ~(f ^ o) & in;
    const int si = sx * RW + (sy >> 6);
    const uint64_t sb = (i == si) ? (1ull << (sy & 63)) : 0ull;
    L.bl[i] = sb;
    L.f0[i] = sb;
    L.m0[i] = 0;
    L.m1[i] = 0;
  }
  __syncthreads();

  // ---- BFS by layers ------------------------------------------------------
  int dstar = -1, end = -1;
  if ((L.tg[sx * RW + (sy >> 6)] >> (sy & 63)) & 1ull) {
    dstar = 0;  // the start cell itself is unexplored
    end = sx * RY + sy;
  } else {
    uint64_t* cur = L.f0;
    uint64_t* nxt = L.f1;
    for (int j = 1; j <= RX * RY; ++j) {
      // slot j % 3 collects layer j; slot (j+1) % 3 is reset for the next
      // layer: every thread has read slot (j-2) % 3 before this layer began
      const int par = j % 3, nxt_slot = (j + 1) % 3;
      if (tid == 0) {
        s_end[nxt_slot] = INT32_MAX;
        s_any[nxt_slot] = 0;
      }
      int any = 0, best = INT32_MAX;
      for (int i = tid; i < NW; i += kDjThreads) {
        const int u = i / RW, w = i - u * RW;
        const uint64_t c = cur[i];
        uint64_t d = c | (c << 1) | (c >> 1);
        if (w > 0) d |= cur[i - 1] >> 63;
        if (w < RW - 1) d |= cur[i + 1] << 63;
        if (u > 0) d |= cur[i - RW];
        if (u < RX - 1) d |= cur[i + RW];
        const uint64_t in = (w == RW - 1) ? last : ~0ull;
        const uint64_t nf = d & ~L.bl[i] & ~L.ob[i] & in;
        nxt[i] = nf;
        if (nf) {
          L.bl[i] |= nf;
          const int m = j % 3;
          if (m == 1) L.m0[i] |= nf;
          if (m == 2) L.m1[i] |= nf;
          any = 1;
          const uint64_t hit = nf & L.tg[i];
          if (hit) best = min(best, u * RY + 64 * w + __ffsll((unsigned long long)hit) - 1);
        }
      }
      if (any) atomicOr(&s_any[par], 1);
      if (best != INT32_MAX) atomicMin(&s_end[par], best);
      __syncthreads();
      if (s_end[par] != INT32_MAX) {
        dstar = j;
        end = s_end[par];
        break;
      }
      if (!s_any[par]) break;  // no reachable unexplored cell: empty path
      uint64_t* t = cur;
      cur = nxt;
      nxt = t;
    }
  }

  // ---- walk back from the end point (first wave, lanes 0..3) --------------
  const int E = s.E, ego = s.ego;
  const int cx0 = sx - ego, cy0 = sy - ego;  // crop origin (dgrid coordinates)
  if (dstar >= 0 && tid < 64) {
    int cu = end / RY, cv = end - (end / RY) * RY;
    int j = dstar;
    const int du = tid == 0 ? 1 : (tid == 1 ? -1 : 0);
    const int dv = tid == 2 ? 1 : (tid == 3 ? -1 : 0);
    for (;;) {
      if (tid == 0) {
        const int r = cu - cx0, c = cv - cy0;
        if (r >= 0 && r < E && c >= 0 && c < E) s_crop[r] |= 1u << c;
      }
      if (j == 0) break;
      const int nu = cu + du, nv = cv + dv;
      bool ok = false;
      if (tid < 4 && nu >= 0 && nu < RX && nv >= 0 && nv < RY) {
        const int i = nu * RW + (nv >> 6), b = nv & 63;
        const int m = (int)((L.m0[i] >> b) & 1ull) + 2 * (int)((L.m1[i] >> b) & 1ull);
        ok = ((L.bl[i] >> b) & 1ull) && m == (j - 1) % 3;
      }
      const uint64_t v = __ballot(ok) & 0xFull;
      if (!v) {  // cannot happen: a cost-j cell has a cost-(j-1) neighbour
        if (tid == 0) atomicOr(s.err, ERR_WINDOW);
        break;
      }
      const int q = __ffsll((unsigned long long)v) - 1;
      cu = __shfl(nu, q);
      cv = __shfl(nv, q);
      --j;
    }
  }
  __syncthreads();
  // ---- obs layer `layer` of agent a: the path cells inside the crop ----------
  uint8_t* dst = obs_out + (((size_t)e * s.N + a) * Lc + layer) * E * E;
  for (int i = tid; i < E * E; i += kDjThreads) {
    const int r = i / E, c = i - r * E;
    dst[i] = (uint8_t)((s_crop[r] >> c) & 1u);
  }
}

// Full-map solve of the listed (env, agent) items: a fixed grid strides over
// the *count entries (the count is uniform, so every wave reaches the end).
// list == nullptr: every (env, agent), one workgroup each.
// count[0] = entries, count[1] = workgroups done: the last workgroup to
// finish zeroes both for the next step's window kernel (every workgroup has
// read the entry count before it counts itself done) and keeps the entry
// count in count[2] (MC_FIELD_DJ_LISTED).
__global__ __launch_bounds__(kDjThreads) void dijkstra_kernel(State s, int pad, int layer, int Lc,
                                                              uint8_t* __restrict__ obs_out,
                                                              const uint32_t* __restrict__ list,
                                                              uint32_t* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t n_items = list ? __atomic_load_n(count, __ATOMIC_RELAXED) : (uint32_t)gridDim.x;
  for (uint32_t it = blockIdx.x; it < n_items; it += (list ? gridDim.x : n_items)) {
    __syncthreads();  // the previous item's LDS reads are done
    const uint32_t ea = list ? list[it] : it;
    dijkstra_full(s, pad, layer, Lc, obs_out, (int)(ea / (uint32_t)s.N), (int)(ea % (uint32_t)s.N),
                  smem);
  }
  if (list && threadIdx.x == 0) {
    if (n_items == 0) {  // nothing listed: nothing to reset (every workgroup read 0)
      if (blockIdx.x == 0) count[2] = 0;
    } else {
      __threadfence();
      if (atomicAdd(count + 1, 1u) == gridDim.x - 1) {
        atomicExch(count + 2, atomicExch(count, 0u));
        atomicExch(count + 1, 0u);
      }
    }
  }
}

// ---- window kernel ---------------------------------------------------------
constexpr int kDjWinDepth = 24;  // BFS layers the 64 x 64 window holds exactly (a multiple of 3)

// whole-wave lane shifts of a 64-bit row (DPP wave_shr:1 / wave_shl:1; the
// lane past the end reads 0): row r - 1 / row r + 1 of the window at lane r
__device__ __forceinline__ uint64_t row_above(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x138, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x138, 0xF, 0xF, true);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t row_below(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, 0x130, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), 0x130, 0xF, 0xF, true);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ uint64_t bits_between(int lo, int hi) {  // bits [lo, hi), 0 <= lo, hi <= 64
  if (hi <= lo) return 0;
  const uint64_t h = hi >= 64 ? ~0ull : ((1ull << hi) - 1);
  return h & ~((1ull << lo) - 1);
}

// bit c of lane `lane`'s row v (lane and c uniform)
__device__ __forceinline__ uint32_t lane_bit(uint64_t v, int lane, int c) {
  const uint32_t w = (uint32_t)(v >> (c & 32));
  return ((uint32_t)__builtin_amdgcn_readlane((int)w, lane) >> (c & 31)) & 1u;
}

// cells whose neighbour at shift S has cost one less (cost mod 3 classes
// K0, K1, K2; the predecessor of class k is class k + 2 mod 3)
__device__ __forceinline__ uint64_t pred(uint64_t k0, uint64_t k1, uint64_t k2, uint64_t s0,
                                         uint64_t s1, uint64_t s2) {
  return (k0 & s2) | (k1 & s0) | (k2 & s1);
}

// grid = B * N workgroups of one wave; lane r holds window row r.  The window
// is tiles [tx - 4, tx + 4) x [ty - 4, ty + 4) of the robot's tile (tx, ty),
// i.e. map rows X0 = 8 (tx - 4) .. X0 + 63 and columns Y0 .. Y0 + 63; bit c of
// a row word is column Y0 + c.  depth: the exact layers (kDjWinDepth).
__global__ __launch_bounds__(64) void dijkstra_window_kernel(State s, int pad, int layer, int Lc,
                                                             uint8_t* __restrict__ obs_out,
                                                             uint32_t* __restrict__ list,
                                                             uint32_t* __restrict__ count,
                                                             int depth) {
  __shared__ uint8_t s_rows[2][64 * 8];  // free / obstacle window rows (tile transpose)
  const uint32_t ea = blockIdx.x;
  const int r = threadIdx.x;
  const int px = s.pos[2 * ea], py = s.pos[2 * ea + 1];  // padded-grid cell of the robot
  const int tx0 = (px >> 3) - 4, ty0 = (py >> 3) - 4;
  const int X0 = 8 * tx0, Y0 = 8 * ty0;
  const int X = X0 + r;
  const int rs = px - X0, cs = py - Y0;  // the robot in window coordinates (32..39)

  // ---- the agent's maps: lane l loads tile (tx0 + l / 8, ty0 + l % 8) of each
  // plane; byte k of it (tile row k) goes to window row 8 (l / 8) + k, byte l % 8
  {
    const int ti = tx0 + (r >> 3), tj = ty0 + (r & 7);
    uint64_t f = 0, o = 0;
    if (ti >= 0 && ti < s.TR && tj >= 0 && tj < s.TC) {
      const size_t i = (size_t)ea * s.MT + tile_index(s.TCS, ti, tj);
      f = s.freem[i];
      o = s.obstm[i];
    }
    uint8_t* df = s_rows[0] + (r >> 3) * 64 + (r & 7);
    uint8_t* dob = s_rows[1] + (r >> 3) * 64 + (r & 7);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      df[8 * k] = (uint8_t)(f >> (8 * k));
      dob[8 * k] = (uint8_t)(o >> (8 * k));
    }
  }
  __syncthreads();
  const uint64_t f = reinterpret_cast<const uint64_t*>(s_rows[0])[r];
  const uint64_t o = reinterpret_cast<const uint64_t*>(s_rows[1])[r];
  // cells of the extended grid (the pad ring is unexplored: a target)
  const uint64_t valid = (X >= -pad && X < s.Wp + pad)
                             ? bits_between(max(-pad - Y0, 0), min(s.Lp + pad - Y0, 64))
                             : 0ull;
  const uint64_t ob = o & ~f & valid;    // g = -1
  const uint64_t tg = ~(f ^ o) & valid;  // g = 0

  // ---- BFS by layers in registers ---------------------------------------------
  // avail: cells not reached yet; m0 / m1: layers j = 1 / 2 (mod 3).  Three
  // layers per trip (each one's mod-3 plane is static) and one target test
  // per trip: a trip with a hit then finds its first layer that has one.
  // Layers past d* (at most two) join the planes too; that is harmless: a
  // neighbour of a cost-j cell has cost j-1, j or j+1, so the walk back's
  // mod-3 test only ever meets those.  A frontier that dies out ends the
  // search at the trip's end (the layers after an empty one are empty).
  // depth is a multiple of 3 (launch_dijkstra).
  int dstar = -1, er = rs, ec = cs;
  bool full = false;
  uint64_t cur = r == rs ? (1ull << cs) : 0ull;
  uint64_t avail = ~ob & valid & ~cur, m0 = 0, m1 = 0;
  if (lane_bit(tg, rs, cs)) {
    dstar = 0;  // the start cell itself is unexplored
  } else {
    for (int j = 0;; j += 3) {
      if (j >= depth) {
        full = true;
        break;
      }
      uint64_t nf[3];
      nf[0] = (cur | (cur << 1) | (cur >> 1) | row_above(cur) | row_below(cur)) & avail;
      avail ^= nf[0];
      m0 |= nf[0];
      nf[1] = (nf[0] | (nf[0] << 1) | (nf[0] >> 1) | row_above(nf[0]) | row_below(nf[0])) & avail;
      avail ^= nf[1];
      m1 |= nf[1];
      nf[2] = (nf[1] | (nf[1] << 1) | (nf[1] >> 1) | row_above(nf[1]) | row_below(nf[1])) & avail;
      avail ^= nf[2];
      cur = nf[2];
      if (__ballot(((nf[0] | nf[1] | nf[2]) & tg) != 0)) {
        // the first layer of the trip with a target; its (x, y)-smallest one:
        // lowest row, then column
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const uint64_t hit = nf[q] & tg;
          const uint64_t hr = __ballot(hit != 0);
          if (hr) {
            er = __ffsll((unsigned long long)hr) - 1;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hit, er);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(hit >> 32), er);
            ec = lo ? __ffs(lo) - 1 : 32 + __ffs(hi) - 1;
            dstar = j + 1 + q;
            break;
          }
        }
        break;
      }
      if (!__ballot(cur != 0)) break;  // no reachable unexplored cell: empty path
    }
  }
  if (full) {  // farther than the window holds: the full kernel solves it
    if (r == 0) list[atomicAdd(count, 1u)] = ea;
    return;
  }

  // ---- walk back (dijkstra.py:166-185): from each cell the first neighbour in
  // the order +x, -x, +y, -y whose cost is one less.  The choice of every
  // reached cell at once, as two direction planes q = 2 d1 + d0 (a reached
  // cell of cost >= 1 always has such a neighbour: its BFS parent); then the
  // walk reads one bit pair per step (readlane, scalar).  Only crop cells are
  // recorded: lane k keeps crop row k.
  const int E = s.E, ego = s.ego;
  const int cr0 = rs - ego, cc0 = cs - ego;  // crop origin (window coordinates)
  uint32_t crop = 0;
  if (dstar >= 0) {
    const uint64_t k1 = m0, k2 = m1, k0 = ~ob & valid & ~avail & ~m0 & ~m1;  // reached, cost = 0 mod 3
    const uint64_t px_ = pred(k0, k1, k2, row_below(k0), row_below(k1), row_below(k2));
    const uint64_t mx_ = pred(k0, k1, k2, row_above(k0), row_above(k1), row_above(k2));
    const uint64_t py_ = pred(k0, k1, k2, k0 >> 1, k1 >> 1, k2 >> 1);
    const uint64_t d1 = ~px_ & ~mx_;
    const uint64_t d0 = (~px_ & mx_) | (d1 & ~py_);
    int cu = er, cv = ec;
    for (int j = dstar;; --j) {
      const int kr = cu - cr0, kc = cv - cc0;
      if ((unsigned)kr < (unsigned)E && (unsigned)kc < (unsigned)E && r == kr) crop |= 1u << kc;
      if (j == 0) break;
      const int q = (int)(2 * lane_bit(d1, cu, cv) + lane_bit(d0, cu, cv));
      cu += q == 0 ? 1 : (q == 1 ? -1 : 0);
      cv += q == 2 ? 1 : (q == 3 ? -1 : 0);
    }
  }
  // ---- obs layer `layer`: crop row k = window row rs - ego + k ------------------
  if (r < E) {
    uint8_t* dst = obs_out + ((size_t)ea * Lc + layer) * E * E + (size_t)r * E;
    for (int c = 0; c < E; ++c) dst[c] = (uint8_t)((crop >> c) & 1u);
  }
}

size_t dijkstra_lds_bytes(const State& s, int pad) {
  const size_t RX = s.Wp + 2 * pad, RW = (s.Lp + 2 * pad + 63) / 64;
  return (7 * RX * RW + 2 * (size_t)s.MT) * 8;
}

// list: u32 [3 + B*N] (entry count, workgroups done, last entry count, then
// the entries),
// library-owned, zero between steps.  window = false: every (env, agent) on
// the full map (the parity tests' second mode).
hipError_t launch_dijkstra(const State& s, int pad, int layer, int Lc, uint8_t* obs,
                           uint32_t* list, bool window, hipStream_t stream) {
  const size_t lds = dijkstra_lds_bytes(s, pad);
  const unsigned items = (unsigned)((size_t)s.B * s.N);
  if (!window) {
    hipLaunchKernelGGL(dijkstra_kernel, dim3(items), dim3(kDjThreads), lds, stream, s, pad, layer,
                       Lc, obs, (const uint32_t*)nullptr, (uint32_t*)nullptr);
    return hipGetLastError();
  }
  static const int depth = [] {  // MARLCOV_DJ_DEPTH: fewer exact layers (diagnostics, A/B)
    const char* v = getenv("MARLCOV_DJ_DEPTH");
    const int d = v ? atoi(v) : kDjWinDepth;
    return d >= 0 && d < kDjWinDepth ? d - d % 3 : kDjWinDepth;  // whole trips of 3 layers
  }();
  hipLaunchKernelGGL(dijkstra_window_kernel, dim3(items), dim3(64), 0, stream, s, pad, layer, Lc,
                     obs, list + 3, list, depth);
  // the listed items: a fixed grid (hipGraph capture) strides over the count
  static const unsigned full_grid = [] {  // MARLCOV_DJ_FULL_GRID: A/B of the fixed grid
    const char* v = getenv("MARLCOV_DJ_FULL_GRID");
    const int g = v ? atoi(v) : 0;
    return g > 0 && g <= 4096 ? (unsigned)g : kDjFullGrid;
  }();
  const unsigned grid = items < full_grid ? items : full_grid;
  hipLaunchKernelGGL(dijkstra_kernel, dim3(grid), dim3(kDjThreads), lds, stream, s, pad, layer, Lc,
                     obs, (const uint32_t*)(list + 3), list);
  return hipGetLastError();
}

}  // namespace mc
