// mc_dist.hip — the dist_reward terms (the C5 frontier reward).
//
// Reference: DecGridRL.get_distance_map dec_grid_rl.py:260-282
//   inv = ~free_pad[i];  d = cv2.distanceTransform(inv, DIST_L1, MASK_PRECISE)
//   d /= max(d) if max(d) > 0;  return 1 - d            (float32 throughout)
// used twice per agent and step:
//   observe() :222-223,239-240  the map BEFORE agent i senses, read at
//             distance_map[x, y] with the post-move (x, y) of the padded grid
//             (no pad offset: a reference quirk, kept) and summed over the
//             agents in float32 into obs_reward;
//   get_egocentric_observations() :350-352  the map AFTER sensing, cropped
//             E x E around the robot into obs layer 3 (float).
// d is the L1 distance of each uncovered cell of the extended grid (padded
// grid + pad ring, dec_grid_rl.py:506-511) to the nearest covered cell; the
// unobstructed L1 distance is the BFS layer index of 4-neighbourhood
// dilations from the covered set.  One workgroup per (env, agent) keeps the
// extended grid as LDS row bitboards (mc_bitboard.h) and runs the layers:
// the last layer index is max(d), and a target cell's d is the layer that
// first reaches it.  OpenCV itself is absent here: the semantics are those of
// the oracle's SciPy restatement (parity vs OpenCV unpinned).
//
// PRE  (before the env kernel): targets are the five cells the robot can end
//      the step on (stay, +x, +y, -x, -y), at the quirk index; out:
//      pre[e][a][0] = max(d), pre[e][a][1 + k] = d of candidate k.
// POST (after it): targets are the E x E crop; out: the float32 obs layer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_bitboard.h"

namespace mc {

namespace {
constexpr int kDtThreads = 256;
constexpr int kMaxTargets = 32 * 32;
}  // namespace

__global__ __launch_bounds__(kDtThreads) void dist_kernel(State s, int pad, int post,
                                                          float* __restrict__ pre_out,
                                                          float* __restrict__ dist_obs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_new[3];
  __shared__ int s_d[kMaxTargets];
  __shared__ int s_cov;
  const int e = blockIdx.x / s.N, a = blockIdx.x - e * s.N;
  const int tid = threadIdx.x;
  const int RX = s.Wp + 2 * pad, RY = s.Lp + 2 * pad, RW = (RY + 63) >> 6, NW = RX * RW;
  uint64_t* R = reinterpret_cast<uint64_t*>(smem);  // reached
  uint64_t* F0 = R + NW;                             // frontier (two buffers)
  uint64_t* F1 = F0 + NW;
  const uint64_t* free_t = s.freem + ((size_t)e * s.N + a) * s.MT;
  const int px = s.pos[((size_t)e * s.N + a) * 2], py = s.pos[((size_t)e * s.N + a) * 2 + 1];

  // targets (extended-grid cells)
  const int E = s.E;
  const int T = post ? E * E : 5;
  for (int t = tid; t < T; t += kDtThreads) s_d[t] = -1;
  if (tid < 3) s_new[tid] = 0;
  if (tid == 0) s_cov = 0;
  __syncthreads();
  const uint64_t last = (RY & 63) ? low_mask(RY & 63) : ~0ull;
  int cov = 0;
  for (int i = tid; i < NW; i += kDtThreads) {
    const int u = i / RW, w = i - u * RW;
    const uint64_t c = row_word(s, free_t, pad, u, w) & ((w == RW - 1) ? last : ~0ull);
    R[i] = c;
    F0[i] = c;
    cov |= c != 0;
  }
  if (cov) atomicOr(&s_cov, 1);
  __syncthreads();

  // target t -> extended cell
  auto target = [&](int t, int& u, int& v) {
    if (post) {
      const int r = t / E, c = t - r * E;
      u = px + pad - s.ego + r;
      v = py + pad - s.ego + c;
    } else {  // distance_map[x, y]: the padded-grid coordinates used as is
      const int dx = t == 1 ? 1 : (t == 3 ? -1 : 0);
      const int dy = t == 2 ? 1 : (t == 4 ? -1 : 0);
      u = px + dx;
      v = py + dy;
    }
  };
  auto reached = [&](const uint64_t* b, int t) -> bool {
    int u, v;
    target(t, u, v);
    if (u < 0 || u >= RX || v < 0 || v >= RY) return false;
    return (b[u * RW + (v >> 6)] >> (v & 63)) & 1ull;
  };

  int M = 0;
  if (!s_cov) {
    // no covered cell: the restatement's convention (-1 everywhere); only the
    // discarded reset-time PRE term can see it
    M = -1;
    for (int t = tid; t < T; t += kDtThreads) s_d[t] = -1;
  } else {
    for (int t = tid; t < T; t += kDtThreads)
      if (reached(R, t)) s_d[t] = 0;
    uint64_t* cur = F0;
    uint64_t* nxt = F1;
    for (int k = 1; k <= RX + RY; ++k) {
      const int slot = k % 3, nslot = (k + 1) % 3;  // see mc_dijkstra.hip
      if (tid == 0) s_new[nslot] = 0;
      int any = 0;
      for (int i = tid; i < NW; i += kDtThreads) {
        const int u = i / RW, w = i - u * RW;
        const uint64_t nf = dilate_word(cur, i, u, w, RX, RW) & ~R[i] & ((w == RW - 1) ? last : ~0ull);
        nxt[i] = nf;
        if (nf) {
          R[i] |= nf;
          any = 1;
        }
      }
      if (any) atomicOr(&s_new[slot], 1);
      __syncthreads();
      if (!s_new[slot]) break;  // every cell reached: max(d) = k - 1
      M = k;
      for (int t = tid; t < T; t += kDtThreads)
        if (s_d[t] < 0 && reached(nxt, t)) s_d[t] = k;
      uint64_t* tmp = cur;
      cur = nxt;
      nxt = tmp;
    }
  }
  __syncthreads();
  const float Mf = (float)M;
  if (post) {
    float* dst = dist_obs + ((size_t)e * s.N + a) * E * E;
    for (int t = tid; t < T; t += kDtThreads) dst[t] = dist_value((float)s_d[t], Mf);
  } else {
    float* dst = pre_out + ((size_t)e * s.N + a) * 8;
    if (tid == 0) dst[0] = Mf;
    if (tid < 5) dst[1 + tid] = (float)s_d[tid];
  }
}

size_t dist_lds_bytes(const State& s, int pad) {
  const size_t RX = s.Wp + 2 * pad, RW = (s.Lp + 2 * pad + 63) / 64;
  return 3 * RX * RW * 8;
}

hipError_t launch_dist(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                       hipStream_t stream) {
  hipLaunchKernelGGL(dist_kernel, dim3((unsigned)((size_t)s.B * s.N)), dim3(kDtThreads),
                     dist_lds_bytes(s, pad), stream, s, pad, post, pre_out, dist_obs);
  return hipGetLastError();
}

}  // namespace mc
