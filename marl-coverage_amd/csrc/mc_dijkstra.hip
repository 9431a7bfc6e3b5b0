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
// GPU form: one workgroup per (env, agent).  The map is held in LDS as row
// bitboards (one bit per cell, 64 columns per word) over the pad-extended
// grid.  BFS layer j is dilate(layer j-1) & ~reached & ~obstacle: a whole
// layer per step of bit operations.  The pop order inside a layer only
// matters for the end point, which is the (x, y)-smallest 0-cell of the first
// layer that holds one — a workgroup min.  For the walk back only cost mod 3
// is kept (two bitboards): a neighbour of a cost-j cell has cost j-1, j or
// j+1, and mod 3 tells them apart.  Four lanes test the four neighbours of
// the walk in parallel; the first valid one in reference order wins.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_bitboard.h"

namespace mc {

namespace {

constexpr int kDjThreads = 256;

struct DjLds {
  uint64_t *ob, *tg, *bl, *f0, *f1, *m0, *m1;
  uint64_t *tf, *to;  // the agent's free / obstacle tiles
};

}  // namespace

// grid = (B * N); block = kDjThreads.  layer: obs layer index written (3).
__global__ __launch_bounds__(kDjThreads) void dijkstra_kernel(State s, int pad, int layer, int Lc,
                                                              uint8_t* __restrict__ obs_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_end[3], s_any[3];  // per BFS layer j: slot j % 3
  __shared__ uint32_t s_crop[32];
  const int e = blockIdx.x / s.N, a = blockIdx.x - e * s.N;
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

size_t dijkstra_lds_bytes(const State& s, int pad) {
  const size_t RX = s.Wp + 2 * pad, RW = (s.Lp + 2 * pad + 63) / 64;
  return (7 * RX * RW + 2 * (size_t)s.MT) * 8;
}

hipError_t launch_dijkstra(const State& s, int pad, int layer, int Lc, uint8_t* obs,
                           hipStream_t stream) {
  const size_t lds = dijkstra_lds_bytes(s, pad);
  hipLaunchKernelGGL(dijkstra_kernel, dim3((unsigned)((size_t)s.B * s.N)), dim3(kDjThreads), lds,
                     stream, s, pad, layer, Lc, obs);
  return hipGetLastError();
}

}  // namespace mc
