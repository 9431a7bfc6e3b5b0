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
                                                          float* __restrict__ dist_obs,
                                                          const uint32_t* __restrict__ list,
                                                          const uint32_t* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_d[kMaxTargets];
  __shared__ int s_cov;
  __shared__ unsigned long long s_key;  // max over the map of (d, distance from the robot, cell)
  __shared__ int s_cpre[kChunks][kStrip], s_csuf[kChunks][kStrip];  // chunk minima per column
  const int tid = threadIdx.x;
  // every map (list == nullptr: one workgroup per (env, agent)), or the maps
  // of a device work list (a fixed grid strides over *count entries: the
  // count is uniform, so every wave reaches the end)
  const uint32_t n_items = list ? *count : (uint32_t)gridDim.x;
  for (uint32_t it = blockIdx.x; it < n_items; it += (list ? gridDim.x : n_items)) {
  const uint32_t ea = list ? list[it] : it;
  const int e = (int)(ea / (uint32_t)s.N), a = (int)(ea - (uint32_t)e * s.N);
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
    s_key = 0;
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
  int vmax = -1, ubest = 0, vbest = 0;  // this thread's first maximum
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
      if (v < RY && d > vmax) {
        vmax = d;
        ubest = u;
        vbest = v;
      }
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
  // witness: of the maxima, the one farthest from the robot (new coverage
  // comes from around the robot, so it keeps M valid longest)
  if (cov && vmax >= 0) {
    const int far = abs(ubest - (px + pad)) + abs(vbest - (py + pad));
    atomicMax(&s_key, ((unsigned long long)vmax << 40) | ((unsigned long long)far << 24) |
                          ((unsigned long long)ubest << 12) | (unsigned long long)vbest);
  }
  __syncthreads();
  // no covered cell: the restatement's convention (-1 everywhere); only the
  // discarded reset-time PRE term can see it
  const int M = cov ? (int)(s_key >> 40) : -1;
  const float Mf = (float)M;
  if (tid == 0) {  // M unknown (-1) while nothing is covered: every step recomputes it
    const int wu = (int)((s_key >> 12) & 0xFFF), wv = (int)(s_key & 0xFFF);
    reinterpret_cast<int2*>(s.dist_mw)[ea] = make_int2(M, pack_witness(wu - pad, wv - pad));
  }
  if (post) {
    float* dst = dist_obs + ((size_t)e * s.N + a) * E * E;
    for (int t = 5 + tid; t < T; t += kDtThreads)
      dst[t - 5] = dist_value((float)(cov ? s_d[t] : -1), Mf);
  }
  float* pd = pre_out + ((size_t)e * s.N + a) * 8;
  if (tid == 0) pd[0] = Mf;
  if (tid < 5) pd[1 + tid] = (float)(cov ? s_d[tid] : -1);
  __syncthreads();  // the LDS is reused by the next item
  }
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
                     dist_lds_bytes(s, pad), stream, s, pad, post, pre_out, dist_obs,
                     (const uint32_t*)nullptr, (const uint32_t*)nullptr);
  return hipGetLastError();
}

// --------------------------------------------------------------------------
// POST terms without a full transform.  Sensing only adds covered cells, so
// d only decreases and max(d) only decreases; the env kernel keeps M
// (S.dist_mw) unless a new cell came closer than M to the witness, a cell
// with d == M (then d(witness) is still M, and no cell exceeds M).  The
// targets (the E x E crop and the 5 end cells of the next step) are near
// the robot, so their d come from a bounded search: a 32 x 32 window
// around the robot, dilated step by step as row bitboards (half a wave per
// map, lane = window row).  d_in(t), the distance to the nearest covered
// cell inside the window, is the true d(t) when d_in(t) <= the distance
// b(t) from t to the nearest cell outside the window (any outside cell is
// at least b(t) away; L1 paths inside a rectangle stay inside it).  A map
// with an unknown M or a target the window cannot settle goes to the work
// list of the full transform.
// --------------------------------------------------------------------------
constexpr int kLocalThreads = 256;
constexpr int kWin = 32;

__global__ __launch_bounds__(kLocalThreads) void dist_local_kernel(State s, int pad,
                                                                   float* __restrict__ pre_out,
                                                                   float* __restrict__ dist_obs,
                                                                   uint32_t* __restrict__ list,
                                                                   uint32_t* __restrict__ count) {
  const int tid = threadIdx.x;
  const uint32_t ea = (blockIdx.x * kLocalThreads + tid) / kWin;
  const int r = tid & (kWin - 1);  // window row of this lane
  const int hb = (tid & 63) & ~(kWin - 1);  // first lane of this half wave
  if (ea >= (uint32_t)s.B * s.N) return;  // whole half waves
  const int2 mw = reinterpret_cast<const int2*>(s.dist_mw)[ea];
  const int M = mw.x;
  const int E = s.E, T = 5 + E * E;
  if (M < 0 || T > kWin) {
    if (r == 0) list[atomicAdd(count, 1u)] = ea;
    return;
  }
  const int2 p = reinterpret_cast<const int2*>(s.pos)[ea];
  const int ti0 = (p.x - 12) >> 3, tj0 = (p.y - 12) >> 3;  // floor: window tile origin
  const int X0 = 8 * ti0, Y0 = 8 * tj0;
  // row r of the window: bits of tiles (ti0 + r/8, tj0 .. tj0 + 3)
  uint32_t cur = 0;
  {
    const int ti = ti0 + (r >> 3);
    const uint64_t* ft = s.freem + (size_t)ea * s.MT;
    if (ti >= 0 && ti < s.TR) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int tj = tj0 + q;
        if (tj >= 0 && tj < s.TC)
          cur |= (uint32_t)((ft[tile_index(s.TCS, ti, tj)] >> (8 * (r & 7))) & 0xFFull) << (8 * q);
      }
    }
  }
  // target of this lane (map coordinates), window-local (tr, tc), bound b
  int tx, ty;
  if (r < 5) {  // distance_map[x, y] of the next step's end cells (quirk: no pad offset)
    tx = p.x + (r == 1 ? 1 : (r == 3 ? -1 : 0)) - pad;
    ty = p.y + (r == 2 ? 1 : (r == 4 ? -1 : 0)) - pad;
  } else {
    const int k = r < T ? r - 5 : 0, rr = k / E;
    tx = p.x - s.ego + rr;
    ty = p.y - s.ego + (k - rr * E);
  }
  const int tr = tx - X0, tc = ty - Y0;
  const bool live = r < T;
  const bool inwin = tr >= 0 && tr < kWin && tc >= 0 && tc < kWin;
  const int b = inwin ? min(min(tr, kWin - 1 - tr), min(tc, kWin - 1 - tc)) + 1 : 0;
  int dt = -1;
  for (int k = 0; k < kWin / 2; ++k) {
    const uint32_t row = (uint32_t)__shfl((int)cur, hb + (inwin ? tr : 0), 64);
    if (live && inwin && dt < 0 && ((row >> tc) & 1u)) dt = k;
    const uint64_t pend = __ballot(live && inwin && dt < 0 && k < b);
    if (((pend >> hb) & 0xFFFFFFFFull) == 0) break;
    const uint32_t up = (uint32_t)__shfl((int)cur, hb + (r > 0 ? r - 1 : 0), 64);
    const uint32_t dn = (uint32_t)__shfl((int)cur, hb + (r < kWin - 1 ? r + 1 : r), 64);
    cur |= (cur << 1) | (cur >> 1) | (r > 0 ? up : 0u) | (r < kWin - 1 ? dn : 0u);
  }
  const bool ok = !live || (inwin && dt >= 0 && dt <= b);
  const uint64_t bad = __ballot(!ok);
  if ((bad >> hb) & 0xFFFFFFFFull) {
    if (r == 0) list[atomicAdd(count, 1u)] = ea;
    return;
  }
  float* pd = pre_out + (size_t)ea * 8;
  if (r == 0) pd[0] = (float)M;
  if (r < 5) pd[1 + r] = (float)dt;
  else if (live) dist_obs[(size_t)ea * E * E + (r - 5)] = dist_value((float)dt, (float)M);
}

// POST: the window search for every map, then the full transform for the
// maps it listed.  The list grid is fixed (hipGraph capture) and strides.
hipError_t launch_dist_post(const State& s, int pad, float* pre_out, float* dist_obs,
                            uint32_t* list, uint32_t* count, hipStream_t stream) {
  const size_t maps = (size_t)s.B * s.N;
  hipError_t err = hipMemsetAsync(count, 0, 4, stream);
  if (err != hipSuccess) return err;
  hipLaunchKernelGGL(dist_local_kernel, dim3((unsigned)((maps * kWin + kLocalThreads - 1) / kLocalThreads)),
                     dim3(kLocalThreads), 0, stream, s, pad, pre_out, dist_obs, list, count);
  err = hipGetLastError();
  if (err != hipSuccess) return err;
  const unsigned grid = (unsigned)(maps < 2048 ? maps : 2048);
  hipLaunchKernelGGL(dist_kernel, dim3(grid), dim3(kDtThreads), dist_lds_bytes(s, pad), stream, s,
                     pad, 1, pre_out, dist_obs, (const uint32_t*)list, (const uint32_t*)count);
  return hipGetLastError();
}

}  // namespace mc
