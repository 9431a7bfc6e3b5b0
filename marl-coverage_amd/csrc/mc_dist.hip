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
// d is the L1 distance of each cell of the extended grid (padded grid + pad
// ring, dec_grid_rl.py:506-511) to the nearest covered (free) cell.  OpenCV
// itself is absent here: the semantics are those of the oracle's SciPy
// restatement (exact integer L1; parity vs OpenCV unpinned).
//
// The L1 transform is separable (Meijster-style):
//   g(u, v) = distance along row u to its nearest covered cell,
//   d(u, v) = min over u' of |u - u'| + g(u', v)
//           = min( u + min_{u'<=u} (g(u',v) - u'),  -u + min_{u'>=u} (g(u',v) + u') ),
// a prefix-min and a suffix-min down every column.  One workgroup per
// (env, agent) walks the extended grid in strips of 32 columns (half a word
// of the LDS row bitboard): the row pass fills a [rows][32] strip of g in
// LDS, the column pass runs the two scans as 8 row chunks per column (a
// chunked parallel scan), and keeps max(d) and the d of the target cells.
// Work is O(cells) per transform, independent of how far the maps are from
// covered (a BFS by layers was O(cells * max d): 6 s per C5 step).
//
// PRE data: for the five cells the robot can end the next step on (stay, +x,
//      +y, -x, -y), at the quirk index: pre[e][a][0] = max(d),
//      pre[e][a][1 + k] = d of candidate k.  Every transform writes it.
// POST (after the env kernel) also writes the E x E crop: the float32 obs
//      layer.  Its PRE data serve the next step, whose sensing starts from
//      these same maps; only map sharing (which changes them at the start of
//      a step) or a state upload makes mc_step run a PRE transform first.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_bitboard.h"

namespace mc {

namespace {
constexpr int kDtThreads = 512;
constexpr int kStrip = 32;                // columns per strip
constexpr int kChunks = kDtThreads / kStrip;  // row chunks per column in the column pass
constexpr int kMaxTargets = 32 * 32;
constexpr int kInf = 1 << 20;             // "no covered cell in this row"
}  // namespace

__global__ __launch_bounds__(kDtThreads) void dist_kernel(State s, int pad, int post,
                                                          float* __restrict__ pre_out,
                                                          float* __restrict__ dist_obs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_d[kMaxTargets];
  __shared__ int s_max, s_cov;
  __shared__ int s_cpre[kChunks][kStrip], s_csuf[kChunks][kStrip];  // chunk minima per column
  const int e = blockIdx.x / s.N, a = blockIdx.x - e * s.N;
  const int tid = threadIdx.x;
  const int RX = s.Wp + 2 * pad, RY = s.Lp + 2 * pad, RW = (RY + 63) >> 6, NW = RX * RW;
  // LDS: C row bitboard [RX][RW] u64 | NL, NR [RX][RW] i32 | G strip [RX][kStrip] u32
  uint64_t* Cb = reinterpret_cast<uint64_t*>(smem);
  int* NL = reinterpret_cast<int*>(Cb + NW);  // last covered column < 64w (or -kInf)
  int* NR = NL + NW;                          // first covered column >= 64(w+1) (or kInf)
  const uint64_t* free_t = s.freem + ((size_t)e * s.N + a) * s.MT;
  const int px = s.pos[((size_t)e * s.N + a) * 2], py = s.pos[((size_t)e * s.N + a) * 2 + 1];
  const int E = s.E;
  // targets: [0, 5) the end cells of the next step (PRE data: the maps do
  // not change between this transform and the next step's sensing unless
  // map sharing runs first), [5, 5 + E*E) the crop (POST only)
  const int T = post ? 5 + E * E : 5;

  // target t -> extended cell (u, v)
  auto target = [&](int t, int& u, int& v) {
    if (t >= 5) {
      const int r = (t - 5) / E, c = (t - 5) - r * E;
      u = px + pad - s.ego + r;
      v = py + pad - s.ego + c;
    } else {  // distance_map[x, y]: the padded-grid coordinates used as is
      const int dx = t == 1 ? 1 : (t == 3 ? -1 : 0);
      const int dy = t == 2 ? 1 : (t == 4 ? -1 : 0);
      u = px + dx;
      v = py + dy;
    }
  };

  for (int t = tid; t < T; t += kDtThreads) s_d[t] = -1;
  if (tid == 0) {
    s_max = 0;
    s_cov = 0;
  }
  const uint64_t last = (RY & 63) ? low_mask(RY & 63) : ~0ull;
  {
    // the agent's tiles into LDS first (coalesced, all loads in flight; the
    // strip area is free until the strips start), then the row bitboard
    uint64_t* tl = reinterpret_cast<uint64_t*>(NL + 2 * NW);
#pragma unroll 4
    for (int i = tid; i < s.MT; i += kDtThreads) tl[i] = free_t[i];
    __syncthreads();
    for (int i = tid; i < NW; i += kDtThreads) {
      const int u = i / RW, w = i - u * RW;
      Cb[i] = row_word(s, tl, pad, u, w) & ((w == RW - 1) ? last : ~0ull);
    }
  }
  __syncthreads();
  // nearest covered column outside each word, per row (one thread per row)
  for (int u = tid; u < RX; u += kDtThreads) {
    int l = -kInf;
    for (int w = 0; w < RW; ++w) {
      NL[u * RW + w] = l;
      const uint64_t c = Cb[u * RW + w];
      if (c) l = 64 * w + 63 - __clzll((long long)c);
    }
    int r = kInf;
    for (int w = RW - 1; w >= 0; --w) {
      NR[u * RW + w] = r;
      const uint64_t c = Cb[u * RW + w];
      if (c) r = 64 * w + __ffsll((unsigned long long)c) - 1;
    }
    if (l != -kInf) atomicOr(&s_cov, 1);
  }
  __syncthreads();
  const bool cov = s_cov != 0;

  // the strips.  G[u][b] packs g (low 16 bits, 0xFFFF = no covered cell in
  // the row) and then the suffix minimum min_{u'>=u} (g(u') + u') (high 16).
  uint32_t* G = reinterpret_cast<uint32_t*>(NR + NW);
  const int col = tid % kStrip, chunk = tid / kStrip;
  const int clen = (RX + kChunks - 1) / kChunks;
  const int u0 = chunk * clen, u1 = min(RX, u0 + clen);
  int vmax = 0;
  for (int st = 0; cov && st < RW * (64 / kStrip); ++st) {
    const int w = st / (64 / kStrip), c0 = st * kStrip;  // word of the strip, first column
    // row pass: g(u, c0 + j) for the strip cells (u, j) = (i / kStrip, i % kStrip)
    for (int i = tid; i < RX * kStrip; i += kDtThreads) {
      const int u = i / kStrip, b = c0 + i % kStrip - 64 * w;  // bit in word w
      const uint64_t c = Cb[u * RW + w];
      const uint64_t le = c & low_mask(b + 1);  // covered at or left of b in the word
      const uint64_t ge = c & ~low_mask(b);     // covered at or right of b
      const int v = 64 * w + b;
      const int left = le ? 64 * w + 63 - __clzll((long long)le) : NL[u * RW + w];
      const int right = ge ? 64 * w + __ffsll((unsigned long long)ge) - 1 : NR[u * RW + w];
      G[i] = (uint32_t)min(min(v - left, right - v), 0xFFFF);
    }
    __syncthreads();
    // column pass: chunk-local minima of g - u and g + u
    int pmin = kInf, smin = kInf;
#pragma unroll 8
    for (int u = u0; u < u1; ++u) {
      const int gv = (int)(G[u * kStrip + col] & 0xFFFFu);
      pmin = min(pmin, gv - u);
      smin = min(smin, gv + u);
    }
    s_cpre[chunk][col] = pmin;
    s_csuf[chunk][col] = smin;
    __syncthreads();
    int pin = kInf, sin_ = kInf;  // minima over the chunks before / after this one
    for (int q = 0; q < chunk; ++q) pin = min(pin, s_cpre[q][col]);
    for (int q = chunk + 1; q < kChunks; ++q) sin_ = min(sin_, s_csuf[q][col]);
    int run = sin_;  // backward sweep: suffix minima into the high half
    for (int u = u1 - 1; u >= u0; --u) {
      const uint32_t gw = G[u * kStrip + col];
      run = min(run, (int)(gw & 0xFFFFu) + u);
      G[u * kStrip + col] = (gw & 0xFFFFu) | ((uint32_t)min(run, 0xFFFF) << 16);
    }
    const int v = c0 + col;
    run = pin;  // forward sweep: d = min(u + prefix, suffix - u), kept in G
    for (int u = u0; u < u1; ++u) {
      const uint32_t gw = G[u * kStrip + col];
      run = min(run, (int)(gw & 0xFFFFu) - u);
      const int d = min(u + run, (int)(gw >> 16) - u);
      if (v < RY) vmax = max(vmax, d);
      G[u * kStrip + col] = (uint32_t)d;
    }
    __syncthreads();
    for (int t = tid; t < T; t += kDtThreads) {
      int tu, tv;
      target(t, tu, tv);
      if (tu >= 0 && tu < RX && tv >= c0 && tv < c0 + kStrip && tv < RY)
        s_d[t] = (int)G[tu * kStrip + (tv - c0)];
    }
    __syncthreads();
  }
  if (cov) atomicMax(&s_max, vmax);
  __syncthreads();
  // no covered cell: the restatement's convention (-1 everywhere); only the
  // discarded reset-time PRE term can see it
  const int M = cov ? s_max : -1;
  const float Mf = (float)M;
  if (post) {
    float* dst = dist_obs + ((size_t)e * s.N + a) * E * E;
    for (int t = 5 + tid; t < T; t += kDtThreads)
      dst[t - 5] = dist_value((float)(cov ? s_d[t] : -1), Mf);
  }
  float* pd = pre_out + ((size_t)e * s.N + a) * 8;
  if (tid == 0) pd[0] = Mf;
  if (tid < 5) pd[1 + tid] = (float)(cov ? s_d[tid] : -1);
}

size_t dist_lds_bytes(const State& s, int pad) {
  const size_t RX = s.Wp + 2 * pad, RW = (s.Lp + 2 * pad + 63) / 64;
  // the strip area also stages the agent's MT tiles before the strips
  const size_t strip = RX * kStrip * 4, tiles = (size_t)s.MT * 8;
  return RX * RW * 8 + 2 * RX * RW * 4 + (strip > tiles ? strip : tiles);
}

hipError_t launch_dist(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                       hipStream_t stream) {
  hipLaunchKernelGGL(dist_kernel, dim3((unsigned)((size_t)s.B * s.N)), dim3(kDtThreads),
                     dist_lds_bytes(s, pad), stream, s, pad, post, pre_out, dist_obs);
  return hipGetLastError();
}

}  // namespace mc
