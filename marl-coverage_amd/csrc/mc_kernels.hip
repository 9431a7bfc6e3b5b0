// mc_kernels.hip — gfx950 kernels of the batched coverage environment.
//
// Hot path restated from ExistentialRobotics/MARL-Coverage
//   Environments/dec_grid_rl.py  DecGridRL.step  :91-169, reset :449-531
//   Environments/Sensors/lidar.py LidarSensor.getMeasurement :16-65
//   Environments/Sensors/squaresensor.py SquareSensor.getMeasurement :15-37
//
// Design (DESIGN.md has the full story):
//   * one workgroup = one env; everything an env step touches is staged in LDS
//     as (2H+1) u64 "window rows" per agent (H = max(ceil(range), egoradius)),
//     so a beam march is an LDS bit test + ds_or_b64 mark per cell;
//   * HBM holds bit-packed per-agent free/obst masks, the union "visited" mask
//     and a 2-plane bit-packed grid (neg = grid<0, pos = grid>0): one step reads
//     and writes only the 2 words per window row that overlap each agent;
//   * moves run sequentially in robot order in wave 0 (one lane per robot,
//     occupancy by ballot) because the reference updates occupancy in place;
//   * the union delta (incremental-coverage reward) is computed without
//     atomics: each touched union word has one owner lane (lowest-index agent
//     whose window covers it) that ORs every agent's new bits for that word;
//   * all float64 arithmetic is the reference's: beam march by sequential
//     += (no FMA possible: adds only), reward assembled in reference order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_internal.h"

namespace mc {

// --------------------------------------------------------------------------
// small helpers
// --------------------------------------------------------------------------
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
    uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint32_t bounded(uint32_t r, uint32_t n) {
  return (uint32_t)(((uint64_t)r * n) >> 32);
}

// Per-workgroup scalars kept in LDS.
struct Scal {
  double pen;          // move penalties, accumulated in robot order
  uint64_t moved;      // robots present in the reference's _robot_pad
  uint32_t cnt_free;   // newly set bits over all agents' free maps
  uint32_t cnt_vis;    // newly covered union cells (the obs reward)
  uint32_t free_old, vis_old;
  int32_t grid;
  int32_t do_reset;
  int32_t currstep;
  int32_t numfree;
  double done_thresh;
  uint32_t ep;         // episode counter of the reset in flight
};
static_assert(sizeof(Scal) <= 64, "Scal must fit the 64-byte LDS block");

struct Lds {
  uint64_t *win_neg, *win_pos, *fpart, *opart, *fwin, *owin, *rawf, *rawo, *rawu;
  int32_t *lx, *ly;
  Scal* sc;
};

__device__ __forceinline__ Lds carve(char* smem, int N, int W) {
  Lds l;
  const int NW = N * W;
  uint64_t* p = reinterpret_cast<uint64_t*>(smem);
  l.win_neg = p;
  l.win_pos = p + NW;
  l.fpart = p + 2 * NW;
  l.opart = p + 3 * NW;
  l.fwin = p + 4 * NW;
  l.owin = p + 5 * NW;
  l.rawf = p + 6 * NW;
  l.rawo = p + 8 * NW;
  l.rawu = p + 10 * NW;
  l.lx = reinterpret_cast<int32_t*>(p + 12 * NW);
  l.ly = l.lx + N;
  l.sc = reinterpret_cast<Scal*>(l.ly + N);  // 12*NW*8 + 8N bytes: 8-aligned
  return l;
}

// Does agent b's staged window cover union word (gx, w)?
__device__ __forceinline__ bool covers(const State& s, const Lds& L, int b, int gx, int w) {
  int dx = gx - L.lx[b];
  if (dx < -s.H || dx > s.H) return false;
  int gy0 = L.ly[b] - s.H;
  int w0 = gy0 >> 6;
  return w == w0 || (w == w0 + 1 && (gy0 & 63) != 0);
}

__device__ __forceinline__ bool owns(const State& s, const Lds& L, int a, int gx, int w) {
  for (int b = 0; b < a; ++b)
    if (covers(s, L, b, gx, w)) return false;
  return true;
}

// --------------------------------------------------------------------------
// stage: bring each agent's window rows of grid / masks / union into LDS.
// With load_masks == false (fresh reset) the masks are known to be zero.
// --------------------------------------------------------------------------
template <int NT>
__device__ void stage(const State& s, const Lds& L, int e, bool load_masks) {
  const int N = s.N, W = s.Wwin, H = s.H, nw = s.nw;
  const uint64_t wmask = low_mask(W);
  const size_t mw = (size_t)s.Wp * nw;
  const int g = L.sc->grid;
  const uint64_t* gn = s.grid_neg + (size_t)g * mw;
  const uint64_t* gp = s.grid_pos + (size_t)g * mw;
  const bool square = s.sensor == 1;
  for (int idx = threadIdx.x; idx < N * W; idx += NT) {
    const int a = idx / W, r = idx - a * W;
    const int gx = L.lx[a] - H + r, gy0 = L.ly[a] - H;
    const int w0 = gy0 >> 6, off = gy0 & 63;
    const bool rowin = gx >= 0 && gx < s.Wp;
    const bool in0 = rowin && w0 >= 0 && w0 < nw;
    const bool in1 = rowin && w0 + 1 >= 0 && w0 + 1 < nw;
    const size_t rb = rowin ? (size_t)gx * nw : 0;
    uint64_t n0 = in0 ? gn[rb + w0] : ~0ull;
    uint64_t n1 = in1 ? gn[rb + w0 + 1] : ~0ull;
    uint64_t p0 = 0, p1 = 0, f0 = 0, f1 = 0, o0 = 0, o1 = 0, u0 = 0, u1 = 0;
    if (square) {
      p0 = in0 ? gp[rb + w0] : 0ull;
      p1 = in1 ? gp[rb + w0 + 1] : 0ull;
    }
    if (load_masks) {
      const size_t base = ((size_t)e * N + a) * mw + rb;
      if (in0) { f0 = s.freem[base + w0]; o0 = s.obstm[base + w0]; }
      if (in1) { f1 = s.freem[base + w0 + 1]; o1 = s.obstm[base + w0 + 1]; }
      const size_t vb = (size_t)e * mw + rb;
      if (in0 && owns(s, L, a, gx, w0)) u0 = s.vis[vb + w0];
      if (in1 && off != 0 && owns(s, L, a, gx, w0 + 1)) u1 = s.vis[vb + w0 + 1];
    }
    L.win_neg[idx] = funnel(n0, n1, off) & wmask;
    L.win_pos[idx] = funnel(p0, p1, off) & wmask;
    L.rawf[2 * idx] = f0;
    L.rawf[2 * idx + 1] = f1;
    L.rawo[2 * idx] = o0;
    L.rawo[2 * idx + 1] = o1;
    L.rawu[2 * idx] = u0;
    L.rawu[2 * idx + 1] = u1;
    L.fwin[idx] = funnel(f0, f1, off) & wmask;
    L.owin[idx] = funnel(o0, o1, off) & wmask;
    L.fpart[idx] = 0;
    L.opart[idx] = 0;
  }
}

// --------------------------------------------------------------------------
// sense: lidar.py:16-65 / squaresensor.py:15-37 into fpart/opart (LDS).
// --------------------------------------------------------------------------
template <int NT>
__device__ void sense(const State& s, const Lds& L) {
  const int N = s.N, W = s.Wwin, H = s.H;
  if (s.sensor == 0) {
    const int nb = s.nbeams;
    const double Wd = (double)s.Wp, Ld = (double)s.Lp;
    const double rng = s.range;
    for (int idx = threadIdx.x; idx < N * nb; idx += NT) {
      const int a = idx / nb, b = idx - a * nb;
      const int x = L.lx[a], y = L.ly[a];
      const double xinc = s.beams[3 * b], yinc = s.beams[3 * b + 1], dinc = s.beams[3 * b + 2];
      double px = (double)x, py = (double)y, dist = 0.0;
      const int ox = x - H, oy = y - H;
      uint64_t* frow = L.fpart + a * W;
      uint64_t* orow = L.opart + a * W;
      const uint64_t* nrow = L.win_neg + a * W;
      // while inbounds and oc[int(cx), int(cy)] >= 0 and currdist < range (lidar.py:52)
      bool inb, clear = false;
      int wr = 0, wc = 0;
      for (int it = 0; it <= H + 2; ++it) {
        inb = px >= 0.0 && py >= 0.0 && px < Wd && py < Ld;
        if (!inb) break;
        wr = (int)px - ox;
        wc = (int)py - oy;
        if ((unsigned)wr >= (unsigned)W || (unsigned)wc >= (unsigned)W) {
          atomicOr(s.err, ERR_WINDOW);
          inb = false;
          break;
        }
        clear = ((nrow[wr] >> wc) & 1ull) == 0ull;
        if (!clear || !(dist < rng)) break;
        atomicOr((unsigned long long*)&frow[wr], 1ull << wc);
        px += xinc;
        py += yinc;
        dist += dinc;
      }
      // final cell (lidar.py:58-63)
      if (inb && clear) {
        atomicOr((unsigned long long*)&frow[wr], 1ull << wc);
      } else if (inb) {
        atomicOr((unsigned long long*)&orow[wr], 1ull << wc);
      } else {
        atomicOr(s.err, ERR_OUT_OF_GRID);
      }
    }
  } else {
    // square window [x-r, x+r] x [y-r, y+r] clamped to the padded grid; the
    // reference overwrites the window with clip(g,0,1)/clip(-g,0,1): on a
    // static grid whose free bits only ever come from clip(g,0,1) this is an
    // OR ("square sensor overwrite").
    const int rr = s.sq_r;
    for (int idx = threadIdx.x; idx < N * W; idx += NT) {
      const int a = idx / W, r = idx - a * W;
      const int gx = L.lx[a] - H + r;
      uint64_t f = 0, o = 0;
      if (r - H >= -rr && r - H <= rr && gx >= 0 && gx < s.Wp) {
        const int gy0 = L.ly[a] - H;
        // window columns c with |c - H| <= rr and 0 <= gy0 + c < Lp
        int c0 = H - rr, c1 = H + rr;
        if (gy0 + c0 < 0) c0 = -gy0;
        if (gy0 + c1 > s.Lp - 1) c1 = s.Lp - 1 - gy0;
        if (c1 >= c0) {
          const uint64_t cm = low_mask(c1 + 1) & ~low_mask(c0);
          f = L.win_pos[idx] & cm;
          o = L.win_neg[idx] & cm;
        }
      }
      L.fpart[idx] = f;
      L.opart[idx] = o;
    }
  }
}

// single_square_tool: the sensor's free result is discarded and only the
// robot's own cell is marked free (dec_grid_rl.py:233-234).
template <int NT>
__device__ void single_tool(const State& s, const Lds& L) {
  const int N = s.N, W = s.Wwin, H = s.H;
  for (int idx = threadIdx.x; idx < N * W; idx += NT) {
    const int r = idx % W;
    L.fpart[idx] = (r == H) ? (1ull << H) : 0ull;
  }
}

// --------------------------------------------------------------------------
// merge: fold fpart/opart into the HBM masks; count new free bits and newly
// covered union cells (dec_grid_rl.py:232-256).
// --------------------------------------------------------------------------
template <int NT>
__device__ void merge(const State& s, const Lds& L, int e) {
  const int N = s.N, W = s.Wwin, H = s.H, nw = s.nw;
  const size_t mw = (size_t)s.Wp * nw;
  uint32_t cf = 0, cv = 0;
  for (int idx = threadIdx.x; idx < N * W; idx += NT) {
    const int a = idx / W, r = idx - a * W;
    const int gx = L.lx[a] - H + r, gy0 = L.ly[a] - H;
    const int w0 = gy0 >> 6, off = gy0 & 63;
    const bool rowin = gx >= 0 && gx < s.Wp;
    const bool in0 = rowin && w0 >= 0 && w0 < nw;
    const bool in1 = rowin && w0 + 1 >= 0 && w0 + 1 < nw && off != 0;
    const uint64_t fp = L.fpart[idx], op = L.opart[idx];
    const uint64_t nf = fp & ~L.fwin[idx];
    const uint64_t no = op & ~L.owin[idx];
    cf += __popcll(nf);
    L.fwin[idx] |= fp;
    L.owin[idx] |= op;
    if (rowin && (nf | no)) {
      const size_t base = ((size_t)e * N + a) * mw + (size_t)gx * nw;
      if (nf) {
        if (in0) s.freem[base + w0] = L.rawf[2 * idx] | (nf << off);
        if (in1) s.freem[base + w0 + 1] = L.rawf[2 * idx + 1] | (nf >> (64 - off));
      }
      if (no) {
        if (in0) s.obstm[base + w0] = L.rawo[2 * idx] | (no << off);
        if (in1) s.obstm[base + w0 + 1] = L.rawo[2 * idx + 1] | (no >> (64 - off));
      }
    }
  }
  // union words: one owner per (row, word); it ORs every covering agent's part
  for (int idx = threadIdx.x; idx < 2 * N * W; idx += NT) {
    const int ia = idx >> 1, k = idx & 1;
    const int a = ia / W, r = ia - a * W;
    const int gx = L.lx[a] - H + r, gy0 = L.ly[a] - H;
    const int w0 = gy0 >> 6, off = gy0 & 63;
    const int w = w0 + k;
    if (gx < 0 || gx >= s.Wp || w < 0 || w >= nw || (k == 1 && off == 0)) continue;
    if (!owns(s, L, a, gx, w)) continue;
    uint64_t contrib = 0;
    for (int b = a; b < N; ++b) {
      if (!covers(s, L, b, gx, w)) continue;
      const int rb = gx - (L.lx[b] - H);
      const int gyb = L.ly[b] - H;
      const int offb = gyb & 63;
      const uint64_t part = L.fpart[b * W + rb];
      contrib |= (w == (gyb >> 6)) ? (part << offb) : (part >> (64 - offb));
    }
    if (contrib) {
      const uint64_t u = L.rawu[idx];
      const uint64_t nn = contrib & ~u;
      if (nn) {
        cv += __popcll(nn);
        s.vis[(size_t)e * mw + (size_t)gx * nw + w] = u | contrib;
      }
    }
  }
  if (cf) atomicAdd(&L.sc->cnt_free, cf);
  if (cv) atomicAdd(&L.sc->cnt_vis, cv);
}

__device__ __forceinline__ bool grid_blocked(const State& s, int g, int x, int y) {
  if (x < 0 || y < 0 || x >= s.Wp || y >= s.Lp) return true;  // isInBounds (:284-295)
  const uint64_t wv = s.grid_neg[((size_t)g * s.Wp + x) * s.nw + (y >> 6)];
  return (wv >> (y & 63)) & 1ull;                               // grid < 0 (:310)
}

// --------------------------------------------------------------------------
// moves: updateRobotPos in robot order (dec_grid_rl.py:128-145, :171-204).
// Wave 0, lane i = robot i.  Occupancy is the live position set, so a robot
// may enter a cell vacated earlier in the same step and is blocked by a
// higher-index robot that has not moved yet (:186,190-199,310).
// --------------------------------------------------------------------------
__device__ void moves(const State& s, const Lds& L, int e, const uint8_t* actions) {
  const int lane = threadIdx.x;  // caller guarantees threadIdx.x < 64
  const int N = s.N;
  const bool live = lane < N;
  int x = live ? L.lx[lane] : INT32_MIN / 2;
  int y = live ? L.ly[lane] : INT32_MIN / 2;
  const int act = live ? (int)actions[(size_t)e * N + lane] : 255;
  const int tx = x + (act == 0) - (act == 2);
  const int ty = y + (act == 1) - (act == 3);
  const int gblk = (live && act < 4) ? (int)grid_blocked(s, L.sc->grid, tx, ty) : 1;
  double pen = 0.0;
  uint64_t moved = L.sc->moved;
  for (int i = 0; i < N; ++i) {
    const int ai = __shfl(act, i);
    if (ai > 3) continue;  // not 0..3: no updateRobotPos call, no penalty
    const int txi = __shfl(tx, i), tyi = __shfl(ty, i), gbi = __shfl(gblk, i);
    const bool occ = __ballot(live && x == txi && y == tyi) != 0ull;
    if (!gbi && !occ) {
      if (lane == i) { x = txi; y = tyi; }
      moved |= 1ull << i;
    } else {
      pen += -s.pen;  // reward += -collision_penalty (:203)
    }
  }
  if (live) { L.lx[lane] = x; L.ly[lane] = y; }
  if (lane == 0) { L.sc->pen = pen; L.sc->moved = moved; }
}

// --------------------------------------------------------------------------
// reset (dec_grid_rl.py:449-531) of env e: pick grid, place robots (injected
// or Philox rejection draw with the reference's acceptance rule), zero the
// maps, then the initial observe() (its reward is discarded, :524).
// --------------------------------------------------------------------------
template <int NT>
__device__ void reset_env(const State& s, const Lds& L, int e, const int32_t* inj_pos) {
  const int N = s.N;
  const int tid = threadIdx.x;
  if (tid == 0) {
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
  // zero this env's maps (:505-514)
  const size_t mw = (size_t)s.Wp * s.nw;
  {
    uint64_t* f = s.freem + (size_t)e * N * mw;
    uint64_t* o = s.obstm + (size_t)e * N * mw;
    for (size_t i = tid; i < (size_t)N * mw; i += NT) { f[i] = 0; o[i] = 0; }
    uint64_t* v = s.vis + (size_t)e * mw;
    for (size_t i = tid; i < mw; i += NT) v[i] = 0;
  }
  if (inj_pos != nullptr) {
    if (tid < N) {
      const int x = inj_pos[((size_t)e * N + tid) * 2];
      const int y = inj_pos[((size_t)e * N + tid) * 2 + 1];
      bool bad = grid_blocked(s, g, x, y);
      for (int j = 0; j < tid; ++j)
        bad |= (inj_pos[((size_t)e * N + j) * 2] == x && inj_pos[((size_t)e * N + j) * 2 + 1] == y);
      if (bad) atomicOr(s.err, ERR_INJECT);
      L.lx[tid] = x;
      L.ly[tid] = y;
    }
  } else if (tid < 64) {
    // x = randint(W), y = randint(L); accept iff grid >= 0 and unoccupied
    // (:491-502).  Candidates are consumed strictly in draw order.
    const int lane = tid;
    int px = INT32_MIN / 2, py = INT32_MIN / 2, placed = 0;
    for (int round = 0; round < 256 && placed < N; ++round) {
      const uint32_t k = (uint32_t)(round * 64 + lane);
      const uint4 r = philox(s.seed, make_uint4(k, (uint32_t)e, ep, 0x706c6163u));
      const int cx = (int)bounded(r.x, (uint32_t)s.Wp);
      const int cy = (int)bounded(r.y, (uint32_t)s.Lp);
      const bool ok = !grid_blocked(s, g, cx, cy);
      uint64_t okm = __ballot(ok);
      while (okm && placed < N) {
        const int j = __ffsll((unsigned long long)okm) - 1;
        okm &= okm - 1;
        const int qx = __shfl(cx, j), qy = __shfl(cy, j);
        const bool clash = __ballot(lane < placed && px == qx && py == qy) != 0ull;
        if (!clash) {
          if (lane == placed) { px = qx; py = qy; }
          ++placed;
        }
      }
    }
    if (placed < N && lane == 0) atomicOr(s.err, ERR_PLACEMENT);
    if (lane < N) { L.lx[lane] = px; L.ly[lane] = py; }
  }
  // the zeroing stores must land before the window stores of merge()
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stage<NT>(s, L, e, /*load_masks=*/false);
  __syncthreads();
  sense<NT>(s, L);
  __syncthreads();
  if (s.sst) { single_tool<NT>(s, L); __syncthreads(); }
  merge<NT>(s, L, e);
  __syncthreads();
  if (tid == 0) {
    s.free_cnt[e] = L.sc->cnt_free;
    s.vis_cnt[e] = L.sc->cnt_vis;
    s.currstep[e] = 0;
  }
}

// --------------------------------------------------------------------------
// the env kernel: one workgroup per env
// --------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void env_kernel(State s, int mode, const uint8_t* __restrict__ actions,
                                                 const uint8_t* __restrict__ env_mask,
                                                 const int32_t* __restrict__ inj_pos,
                                                 double* __restrict__ reward_out,
                                                 uint8_t* __restrict__ done_out,
                                                 uint8_t* __restrict__ obs_out,
                                                 uint8_t* __restrict__ adj_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int e = blockIdx.x;
  const int tid = threadIdx.x;
  const int N = s.N, W = s.Wwin, H = s.H;
  const Lds L = carve(smem, N, W);

  const bool is_step = mode == MODE_STEP;
  const bool sentinel = is_step && actions[(size_t)e * N] == 255;
  const bool reset_req = !is_step && (env_mask == nullptr || env_mask[e] != 0);
  const bool active_step = is_step && !sentinel;

  if (tid == 0) {
    const int g = s.env_grid[e];
    L.sc->grid = g;
    L.sc->moved = s.moved[e];
    L.sc->pen = 0.0;
    L.sc->cnt_free = 0;
    L.sc->cnt_vis = 0;
    L.sc->do_reset = 0;
    if (active_step) {
      L.sc->free_old = s.free_cnt[e];
      L.sc->vis_old = s.vis_cnt[e];
      L.sc->currstep = s.currstep[e];
      L.sc->done_thresh = s.done_thresh[e];
      L.sc->numfree = s.numfree[g];
    }
  }
  if (tid < N) {
    L.lx[tid] = s.pos[((size_t)e * N + tid) * 2];
    L.ly[tid] = s.pos[((size_t)e * N + tid) * 2 + 1];
  }
  __syncthreads();

  if (active_step) {
    if (tid < 64) moves(s, L, e, actions);
    __syncthreads();
    stage<NT>(s, L, e, true);
    __syncthreads();
    sense<NT>(s, L);
    __syncthreads();
    if (s.sst) { single_tool<NT>(s, L); __syncthreads(); }
    merge<NT>(s, L, e);
    __syncthreads();
    if (tid == 0) {
      Scal* c = L.sc;
      const uint32_t fc = c->free_old + c->cnt_free;
      const uint32_t vc = c->vis_old + c->cnt_vis;
      const int cs = c->currstep + 1;                            // :154
      double r = c->pen;                                         // :120,132-145
      r += (double)c->cnt_vis;                                   // :151, :256
      const double pc = (double)fc / (double)c->numfree;         // :552
      double dt = c->done_thresh;
      const double thr = (1.0 < dt) ? 1.0 : dt;                  // min(done_thresh, 1)
      const bool covered = thr <= pc;
      if (covered) r += s.term;                                  // :156-157
      bool done = false;
      if (covered) { dt += s.dincr; done = true; }               // :540-543
      else if (cs == s.maxsteps) done = true;                    // :544-545
      reward_out[e] = r;
      done_out[e] = done ? 1 : 0;
      s.free_cnt[e] = fc;
      s.vis_cnt[e] = vc;
      s.currstep[e] = cs;
      s.done_thresh[e] = dt;
      c->do_reset = (done && s.auto_reset) ? 1 : 0;
    }
    __syncthreads();
    if (L.sc->do_reset) {
      reset_env<NT>(s, L, e, nullptr);
      __syncthreads();
    }
  } else if (reset_req) {
    reset_env<NT>(s, L, e, inj_pos);
    __syncthreads();
  } else {
    // sentinel step / untouched env in a partial reset: observations of the
    // current state only (dec_grid_rl.py:104-107,160)
    stage<NT>(s, L, e, true);
    __syncthreads();
    if (tid == 0 && sentinel) {
      reward_out[e] = 0.0;
      done_out[e] = 1;
    }
  }

  const bool changed = active_step || reset_req || L.sc->do_reset;
  if (changed) {
    if (tid < N) {
      s.pos[((size_t)e * N + tid) * 2] = L.lx[tid];
      s.pos[((size_t)e * N + tid) * 2 + 1] = L.ly[tid];
    }
    if (tid == 0) s.moved[e] = L.sc->moved;
  }

  // egocentric observations (dec_grid_rl.py:312-372): layer 0 robot_pad,
  // layer 1 own free map, layer 2 own obstacle map, E x E around the robot.
  const int E = s.E, EE = E * E, per = s.Lc * EE, ego = s.ego;
  uint8_t* o = obs_out + (size_t)e * N * per;
  const uint64_t moved = L.sc->moved;
  for (int idx = tid; idx < N * per; idx += NT) {
    const int a = idx / per, rem = idx - a * per;
    const int layer = rem / EE, cell = rem - layer * EE;
    const int rr = cell / E, cc = cell - rr * E;
    uint8_t v = 0;
    if (layer == 0) {
      const int cx = L.lx[a] - ego + rr, cy = L.ly[a] - ego + cc;
      for (uint64_t m = moved; m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        if (L.lx[j] == cx && L.ly[j] == cy) v = 1;
      }
    } else if (layer == 1) {
      v = (uint8_t)((L.fwin[a * W + rr + H - ego] >> (cc + H - ego)) & 1ull);
    } else if (layer == 2) {
      v = (uint8_t)((L.owin[a * W + rr + H - ego] >> (cc + H - ego)) & 1ull);
    }
    o[idx] = v;
  }
  if (adj_out != nullptr) {  // updateCommmunicationGraph (:374-391)
    uint8_t* ad = adj_out + (size_t)e * N * N;
    for (int idx = tid; idx < N * N; idx += NT) {
      const int i = idx / N, j = idx - i * N;
      const int dx = abs(L.lx[i] - L.lx[j]), dy = abs(L.ly[i] - L.ly[j]);
      ad[idx] = (max(dx, dy) <= s.comm_r) ? 1 : 0;
    }
  }
}

// --------------------------------------------------------------------------
// shareMaps (dec_grid_rl.py:423-447), run before the step kernel when
// map_sharing is on: agent i's maps <- OR over {j: adj(i,j) or i==j}, with
// adj from the positions at the start of the step (the last comm graph).
// grid = (ceil(Wp*nw / 64), B); block = 64 lanes, one word position each.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(64) void share_kernel(State s, const uint8_t* __restrict__ actions) {
  const int e = blockIdx.y;
  const int N = s.N;
  if (actions[(size_t)e * N] == 255) return;  // sentinel: no state change
  const size_t mw = (size_t)s.Wp * s.nw;
  const size_t w = (size_t)blockIdx.x * 64 + threadIdx.x;
  __shared__ int32_t px[64], py[64];
  if (threadIdx.x < N) {
    px[threadIdx.x] = s.pos[((size_t)e * N + threadIdx.x) * 2];
    py[threadIdx.x] = s.pos[((size_t)e * N + threadIdx.x) * 2 + 1];
  }
  __syncthreads();
  if (w >= mw) return;
  uint64_t* f = s.freem + (size_t)e * N * mw + w;
  uint64_t* o = s.obstm + (size_t)e * N * mw + w;
  uint64_t fold[64], oold[64];
  for (int j = 0; j < N; ++j) { fold[j] = f[j * mw]; oold[j] = o[j * mw]; }
  uint32_t cnt = 0;
  for (int i = 0; i < N; ++i) {
    uint64_t fn = 0, on = 0;
    for (int j = 0; j < N; ++j) {
      const int d = max(abs(px[i] - px[j]), abs(py[i] - py[j]));
      if (d <= s.comm_r || i == j) { fn |= fold[j]; on |= oold[j]; }
    }
    cnt += __popcll(fn & ~fold[i]);
    if (fn != fold[i]) f[i * mw] = fn;
    if (on != oold[i]) o[i * mw] = on;
  }
  if (cnt) atomicAdd(&s.free_cnt[e], cnt);
}

// --------------------------------------------------------------------------
// grid pool upload / generation
// --------------------------------------------------------------------------
// int8 [G][Wp][Lp] -> neg/pos bit planes, numfree[g] = count(grid > 0).
__global__ void pack_grids_kernel(State s, const int8_t* __restrict__ grids) {
  const size_t mw = (size_t)s.Wp * s.nw;
  const size_t total = (size_t)s.G * mw;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int g = (int)(i / mw);
    const size_t rem = i - (size_t)g * mw;
    const int x = (int)(rem / s.nw), w = (int)(rem - (size_t)x * s.nw);
    const int8_t* row = grids + ((size_t)g * s.Wp + x) * s.Lp;
    uint64_t neg = 0, pos = 0;
    for (int b = 0; b < 64; ++b) {
      const int y = w * 64 + b;
      if (y >= s.Lp) { neg |= 1ull << b; continue; }
      const int8_t v = row[y];
      if (v < 0) neg |= 1ull << b;
      if (v > 0) pos |= 1ull << b;
    }
    const_cast<uint64_t*>(s.grid_neg)[i] = neg;
    const_cast<uint64_t*>(s.grid_pos)[i] = pos;
    if (pos) atomicAdd(const_cast<int32_t*>(&s.numfree[g]), (int32_t)__popcll(pos));
  }
}

// Bernoulli(p) obstacles in the interior, -1 border (gridgen semantics,
// Utils/gridmaker.py:127-128, plus the np.pad of dec_grid_rl.py:471).
__global__ void gen_grids_kernel(State s, uint64_t seed, uint32_t thresh, int all_free) {
  const size_t mw = (size_t)s.Wp * s.nw;
  const size_t total = (size_t)s.G * mw;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int g = (int)(i / mw);
    const size_t rem = i - (size_t)g * mw;
    const int x = (int)(rem / s.nw), w = (int)(rem - (size_t)x * s.nw);
    uint64_t neg = 0;
    for (int q = 0; q < 16; ++q) {
      const uint4 r = philox(seed, make_uint4((uint32_t)g, (uint32_t)x, (uint32_t)(w * 16 + q), 0x67656e21u));
      const uint32_t rv[4] = {r.x, r.y, r.z, r.w};
      for (int t = 0; t < 4; ++t) {
        const int b = q * 4 + t;
        const int y = w * 64 + b;
        const bool border = x == 0 || x == s.Wp - 1 || y == 0 || y >= s.Lp - 1;
        if (border || (!all_free && rv[t] < thresh)) neg |= 1ull << b;
      }
    }
    const uint64_t valid = (w == s.nw - 1 && (s.Lp & 63)) ? low_mask(s.Lp & 63) : ~0ull;
    const uint64_t pos = ~neg & valid;
    const_cast<uint64_t*>(s.grid_neg)[i] = neg;
    const_cast<uint64_t*>(s.grid_pos)[i] = pos;
    if (pos) atomicAdd(const_cast<int32_t*>(&s.numfree[g]), (int32_t)__popcll(pos));
  }
}

// --------------------------------------------------------------------------
// host-side launchers (called from mc_capi.hip)
// --------------------------------------------------------------------------
hipError_t launch_env(const State& s, int mode, const uint8_t* actions, const uint8_t* env_mask,
                      const int32_t* inj_pos, double* reward, uint8_t* done, uint8_t* obs,
                      uint8_t* adj, int nt, hipStream_t stream) {
  const size_t lds = env_kernel_lds_bytes(s.N, s.Wwin);
  dim3 grid(s.B), block(nt);
  switch (nt) {
    case 64:
      hipLaunchKernelGGL((env_kernel<64>), grid, block, lds, stream, s, mode, actions, env_mask,
                         inj_pos, reward, done, obs, adj);
      break;
    case 128:
      hipLaunchKernelGGL((env_kernel<128>), grid, block, lds, stream, s, mode, actions, env_mask,
                         inj_pos, reward, done, obs, adj);
      break;
    case 256:
      hipLaunchKernelGGL((env_kernel<256>), grid, block, lds, stream, s, mode, actions, env_mask,
                         inj_pos, reward, done, obs, adj);
      break;
    default:
      hipLaunchKernelGGL((env_kernel<512>), grid, block, lds, stream, s, mode, actions, env_mask,
                         inj_pos, reward, done, obs, adj);
      break;
  }
  return hipGetLastError();
}

hipError_t launch_share(const State& s, const uint8_t* actions, hipStream_t stream) {
  const size_t mw = (size_t)s.Wp * s.nw;
  dim3 grid((unsigned)((mw + 63) / 64), s.B), block(64);
  hipLaunchKernelGGL(share_kernel, grid, block, 0, stream, s, actions);
  return hipGetLastError();
}

hipError_t launch_pack(const State& s, const int8_t* grids, hipStream_t stream) {
  const size_t total = (size_t)s.G * s.Wp * s.nw;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(pack_grids_kernel, dim3(blocks), dim3(256), 0, stream, s, grids);
  return hipGetLastError();
}

hipError_t launch_gen(const State& s, uint64_t seed, double p, hipStream_t stream) {
  const size_t total = (size_t)s.G * s.Wp * s.nw;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  double t = p * 4294967296.0;
  uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (t <= 0.0 ? 0u : (uint32_t)t);
  hipLaunchKernelGGL(gen_grids_kernel, dim3(blocks), dim3(256), 0, stream, s, seed, thresh,
                     p <= 0.0 ? 1 : 0);
  return hipGetLastError();
}

}  // namespace mc
