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
// a prefix-min and a suffix-min down every column.  One workgroup per map
// walks the extended grid in strips of 32 columns:
//   row pass    a thread per row computes the strip's 32 g in registers (two
//               bit scans with the nearest covered column left / right of the
//               strip carried in registers) and writes them as u16 to LDS;
//   column pass a thread per (column, chunk of kCL rows) loads its g into
//               registers, publishes the chunk's minima of g - u and g + u,
//               and after one barrier finishes both scans in registers
//               (chunked parallel scan: no LDS latency inside the scans).
// Work is O(cells) per transform; LDS holds the row bitboard and one u16
// strip (~78 KB at C5: two workgroups per CU).
//
// PRE data: for the five cells the robot can end the next step on (stay, +x,
//      +y, -x, -y), at the quirk index: pre[e][a][0] = max(d),
//      pre[e][a][1 + k] = d of candidate k.  Every transform writes it.
// POST also writes the E x E crop: the float32 obs layer.  Its PRE data serve
//      the next step, whose sensing starts from these same maps; only map
//      sharing (which changes them at the start of a step) or a state upload
//      makes mc_step run a PRE transform first.
// Every transform also leaves (M, witness) for the incremental path below.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mc_bitboard.h"

namespace mc {

// -DMC_DIST_STAMPS diagnostic builds (tools/dist_stamps.py): per listed map
// ea (< B * 16) one u64 in State::stamps -- cycles/16 of the staging + fast
// path, the main strips and the cache pass (16 bits each), and flags (bit 48
// fast path served, 49 one-pass cache list kept, 50 second cache pass ran).
#ifdef MC_DIST_STAMPS
#define DSTAMP(v)                                                               \
  do {                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                          \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                          \
  } while (0)
#else
#define DSTAMP(v) \
  do {            \
  } while (0)
#endif

namespace {
#ifndef MC_DT_THREADS  // build knob (A/B): threads per transform workgroup, 512 or 1024
#define MC_DT_THREADS 512
#endif
constexpr int kDtThreads = MC_DT_THREADS;
static_assert(kDtThreads == 512 || kDtThreads == 1024, "a column pair's chunks are a half wave or a wave");
constexpr int kStrip = 32;                     // columns per strip
constexpr int kPairs = kStrip / 2;             // column pairs (packed u16 halves) per strip
constexpr int kCh = kDtThreads / kPairs;       // row chunks per column pair: the lanes of a half wave / a wave
// LDS stride, padded off the bank period.  512 threads: a strip row is 36
// u16 (72 B = 18 dwords: the row pass's 8-byte stores of 16 consecutive rows
// hit 32 distinct banks; at 64 B four rows shared each bank; the column
// pass's dword reads of 32 chunks 17 rows apart hit 32 distinct banks).
// 1024 threads: 34 u16 (17 dwords, odd: 32 chunks 9 rows apart, and 16
// consecutive rows' 8-byte stores, on distinct banks)
constexpr int kSP = kCh == 64 ? 34 : 36;
constexpr int kInf = 1 << 20;                  // "no covered cell in this row"
constexpr int kMaxRows = 832;                  // RX limit of the largest instantiation
constexpr int kRowOff = 1024;                  // g - u + kRowOff > 0 (u < kMaxRows)
constexpr int kMaxTrack = kDistStrips;         // strips whose max(d) the cache pass can skip by
#ifndef MC_DIST_ONEPASS  // build knob (A/B): collect the cache cells in the transform pass
#define MC_DIST_ONEPASS 1
#endif
constexpr bool kOnePass = MC_DIST_ONEPASS != 0;
#ifndef MC_FAST_TILES  // build knob (A/B): tiles the cache fast path stages (box + 25 around the robot)
// (1024 since round 5: 8 KB of LDS, more workgroups per CU; a box past it
// sends the map to the full transform.  At the C5 steady state and early
// phase the served counts were unchanged, profiles/r5/fast2/)
#define MC_FAST_TILES 1024
#endif
constexpr int kFastTiles = MC_FAST_TILES;
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
constexpr u16x2 kNone2 = {0xFFFF, 0xFFFF};
constexpr u16x2 kRowOff2 = {kRowOff, kRowOff};
__device__ __forceinline__ u16x2 splat2(int v) { return u16x2{(uint16_t)v, (uint16_t)v}; }

// The thread index as an opaque value: the compiler can neither hoist what
// is derived from it out of the item loops nor keep it live across them (it
// hoisted every per-thread address and lane mask of an item out of
// dist_kernel_t's item loop and spilled them: 24 VGPRs at <17>, round 5)
__device__ __forceinline__ int opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// Packed minima across the 32 chunks of a column pair (lane c of a half wave
// = chunk c): over the chunks before this one / after it (0xFFFF: none).
// DPP row shifts inside each 16-lane row, the other row's total by readlane.
template <int CTRL>
__device__ __forceinline__ u16x2 dpp2(u16x2 v) {  // source lane out of the row: 0xFFFF pair
  return __builtin_bit_cast(u16x2, __builtin_amdgcn_update_dpp((int)0xFFFFFFFF, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, false));
}
// 64 chunks (1024 threads): the whole wave, four 16-lane rows
__device__ __forceinline__ u16x2 excl_prefix_min64(u16x2 v) {
  const int l = opaque_tid() & 63;
  u16x2 x = __builtin_elementwise_min(v, dpp2<0x111>(v));
  x = __builtin_elementwise_min(x, dpp2<0x112>(x));
  x = __builtin_elementwise_min(x, dpp2<0x114>(x));
  x = __builtin_elementwise_min(x, dpp2<0x118>(x));  // inclusive within the row
  const u16x2 t0 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 15));
  const u16x2 t1 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 31));
  const u16x2 t2 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 47));
  const u16x2 c1 = t0, c2 = __builtin_elementwise_min(t0, t1), c3 = __builtin_elementwise_min(c2, t2);
  const int row = l >> 4;
  const u16x2 carry = row == 0 ? kNone2 : (row == 1 ? c1 : (row == 2 ? c2 : c3));  // the rows before
  u16x2 e = dpp2<0x111>(x);
  e = (l & 15) == 0 ? kNone2 : e;
  return __builtin_elementwise_min(e, carry);
}
__device__ __forceinline__ u16x2 excl_suffix_min64(u16x2 v) {
  const int l = opaque_tid() & 63;
  u16x2 x = __builtin_elementwise_min(v, dpp2<0x101>(v));
  x = __builtin_elementwise_min(x, dpp2<0x102>(x));
  x = __builtin_elementwise_min(x, dpp2<0x104>(x));
  x = __builtin_elementwise_min(x, dpp2<0x108>(x));  // inclusive within the row, from the right
  const u16x2 s1 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 16));
  const u16x2 s2 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 32));
  const u16x2 s3 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 48));
  const u16x2 c2 = s3, c1 = __builtin_elementwise_min(s2, s3), c0 = __builtin_elementwise_min(c1, s1);
  const int row = l >> 4;
  const u16x2 carry = row == 3 ? kNone2 : (row == 2 ? c2 : (row == 1 ? c1 : c0));  // the rows after
  u16x2 e = dpp2<0x101>(x);
  e = (l & 15) == 15 ? kNone2 : e;
  return __builtin_elementwise_min(e, carry);
}
__device__ __forceinline__ u16x2 excl_prefix_min32(u16x2 v) {
  const int l = opaque_tid() & 63;
  u16x2 x = __builtin_elementwise_min(v, dpp2<0x111>(v));  // row_shr:1
  x = __builtin_elementwise_min(x, dpp2<0x112>(x));        // row_shr:2
  x = __builtin_elementwise_min(x, dpp2<0x114>(x));        // row_shr:4
  x = __builtin_elementwise_min(x, dpp2<0x118>(x));        // row_shr:8: inclusive within the row
  const u16x2 r0 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 15));
  const u16x2 r2 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 47));
  const u16x2 carry = (l & 16) ? ((l & 32) ? r2 : r0) : kNone2;  // rows 1, 3: the row before
  u16x2 e = dpp2<0x111>(x);                                     // exclusive within the row
  e = (l & 15) == 0 ? kNone2 : e;
  return __builtin_elementwise_min(e, carry);
}
__device__ __forceinline__ u16x2 excl_suffix_min32(u16x2 v) {
  const int l = opaque_tid() & 63;
  u16x2 x = __builtin_elementwise_min(v, dpp2<0x101>(v));  // row_shl:1
  x = __builtin_elementwise_min(x, dpp2<0x102>(x));        // row_shl:2
  x = __builtin_elementwise_min(x, dpp2<0x104>(x));        // row_shl:4
  x = __builtin_elementwise_min(x, dpp2<0x108>(x));        // row_shl:8
  const u16x2 r1 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 16));
  const u16x2 r3 = __builtin_bit_cast(u16x2, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 48));
  const u16x2 carry = (l & 16) ? kNone2 : ((l & 32) ? r3 : r1);  // rows 0, 2: the row after
  u16x2 e = dpp2<0x101>(x);
  e = (l & 15) == 15 ? kNone2 : e;
  return __builtin_elementwise_min(e, carry);
}
// L1 distance from cell (cx, cy) to the nearest set bit of tile nb (origin
// (x0, y0)), or cap when none is nearer (the tile-box bound first)
__device__ __forceinline__ int tile_min_dist(uint64_t nb, int x0, int y0, int cx, int cy, int cap) {
  const int bx = max(0, max(x0 - cx, cx - (x0 + 7)));
  const int by = max(0, max(y0 - cy, cy - (y0 + 7)));
  if (!nb || bx + by >= cap) return cap;
  const int p = cy - y0;  // the cell's column relative to the tile
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)(nb >> (8 * r)) & 0xFFu;
    if (!row) continue;
    int dy;
    if (p < 0) dy = __ffs(row) - 1 - p;
    else if (p > 7) dy = p - (31 - __clz(row));
    else {
      const uint32_t lo = row & ((2u << p) - 1u), hi = row >> p;
      dy = lo ? p - (31 - __clz(lo)) : 8;
      if (hi) dy = min(dy, __ffs(hi) - 1);
    }
    cap = min(cap, abs(x0 + r - cx) + dy);
  }
  return cap;
}

// |c - the nearest set bit of row| (0 <= c < 64), or kInf for an empty row
__device__ __forceinline__ int row_near(uint64_t row, int c) {
  const uint64_t lo = row & ((2ull << c) - 1ull), hi = row >> c;  // (c = 63: 2 << 63 wraps to 0, lo = row)
  int h = kInf;
  if (lo) h = c - (63 - __clzll((unsigned long long)lo));
  if (hi) h = min(h, __ffsll((unsigned long long)hi) - 1);
  return h;
}

// Hand-off between the parts of a split map inside one launch (the fused
// mode 2, MI355X_MICROARCH.md: the fan-in row of the hand-off table): the
// parts store the handed-off words `sc1` (agent-scope relaxed atomic stores
// lower to global_store ... sc1: write-through past the XCD's L2), every
// storing wave waits for its stores, and after a workgroup barrier one lane
// adds to the map's counter (agent scope); the part whose add returns S - 1
// loads them back `sc1` (global_load ... sc1: past its L1).  Global address
// space casts keep them global_ (never flat_) instructions.
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) { st_sc1(reinterpret_cast<uint32_t*>(p), __float_as_uint(v)); }
__device__ __forceinline__ void st_sc1(int2* p, int2 v) {
  __hip_atomic_store((g_u64*)p, (unsigned long long)(uint32_t)v.x | ((unsigned long long)(uint32_t)v.y << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load((g_u32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) { return __uint_as_float(ld_sc1(reinterpret_cast<const uint32_t*>(p))); }
__device__ __forceinline__ unsigned long long ld_sc1(const unsigned long long* p) {
  return __hip_atomic_load((g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int2 ld_sc1(const int2* p) {
  const unsigned long long v = ld_sc1(reinterpret_cast<const unsigned long long*>(p));
  return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
}
// plain or `sc1`
template <typename T>
__device__ __forceinline__ T ld_ho(const T* p, bool sc1) { return sc1 ? ld_sc1(p) : *p; }
template <typename T>
__device__ __forceinline__ void st_ho(T* p, T v, bool sc1) {
  if (sc1) st_sc1(p, v);
  else *p = v;
}

// max over the wave (every lane gets it)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return v;
}

// The env kernel's work list: kListShards shards of s.dist_cap entries
// (State::dist_shc), read as one list of pre[kListShards] entries in shard
// order.  The counts were written by an earlier launch: plain loads.
struct ListView {
  uint32_t pre[kListShards + 1];  // entries before shard k
};
__device__ __forceinline__ ListView list_view(const State& s) {
  ListView v;
  v.pre[0] = 0;
#pragma unroll
  for (int k = 0; k < kListShards; ++k) v.pre[k + 1] = v.pre[k] + s.dist_shc[k * kShardStride];
  return v;
}
__device__ __forceinline__ uint32_t list_entry(const State& s, const ListView& v, const uint32_t* list, uint32_t i) {
  uint32_t off = i;
#pragma unroll
  for (int k = 1; k < kListShards; ++k) off = i >= v.pre[k] ? (uint32_t)k * s.dist_cap + (i - v.pre[k]) : off;
  return list[off];
}
}  // namespace

// rows per column chunk: the instantiation (8, 17 or 26) whose kCh chunks
// cover RX; the strip holds kCh * chunk rows (rows >= RX are padding with
// no covered cell)
__host__ __device__ constexpr int chunk_rows(int RX) {
  return kCh == 64 ? (RX <= 256 ? 4 : (RX <= 576 ? 9 : 13)) : (RX <= 256 ? 8 : (RX <= 544 ? 17 : 26));
}

// LDS carve of the full transform (bytes): row bitboard | strip (u16, also the
// tile staging area) | chunk minima | targets
struct DtLds {
  size_t cb, strip, mins, tgt, total;
};
__host__ __device__ inline DtLds dt_lds(int RX, int RY, int MT, int T) {
  DtLds L;
  const int RW = (RY + 63) >> 6;
  L.cb = (size_t)RX * RW * 8;
  // the strip area also holds the map's rows while the row bitboard is built
  // (at most RX x RW words)
  const size_t st = (size_t)kCh * chunk_rows(RX) * kSP * 2, tiles = (size_t)RX * RW * 8;
  L.strip = ((st > tiles ? st : tiles) + 15) & ~(size_t)15;
  L.mins = 0;
  L.tgt = ((size_t)T * 4 + 15) & ~(size_t)15;
  L.total = L.cb + L.strip + L.mins + L.tgt;
  return L;
}

// ---- the top-cell cache fast path of one listed map: the cells covered
// since the cached d were exact all lie in the box, so the current d of a
// cached cell is min(its d, the distance to the box's covered cells).  Every
// other cell had d < M0 - kDistT when the cache was taken, and d only
// decreases: if some cached cell still has d >= M0 - kDistT, the largest such
// d is max(d) and that cell a witness.  The targets (all within a few cells
// of the robot, whose own cell is covered) come from the 5 x 5 tiles around
// them.  NTH threads; stages the box tiles into ft (kFastTiles words),
// leaves the cells' new d in cdv, the targets' d in s_d (-1 stays: none),
// the best (d << 16 | index) in *fkey and a target the 40 x 40 block cannot
// settle in *ffail; `tried` = false when the box is too large to stage.
// `span` (optional, 6 * kSpan words): the staged box's covered extent per
// row and per column and their 1D transforms, for the cells outside the
// box's column or row band.
// Ends with a barrier.
constexpr int kSpan = 256;  // box rows / columns the span arrays hold
template <int NTH>
__device__ __forceinline__ void cache_try(const State& s, int pad, int T, int px, int py, const uint64_t* free_t,
                                          int ccnt, int bx0, int by0, int bx1, int by1, uint64_t* ft,
                                          const int32_t* cc, const int32_t* cd, uint16_t* cdv, int* s_d,
                                          uint32_t* fkey, int* ffail, bool& tried, uint32_t* span = nullptr,
                                          uint64_t* ts = nullptr) {
  const int tid = opaque_tid(), E = s.E;
  const int ti0 = bx0 >> 3, ti1 = bx1 >> 3, tj0 = by0 >> 3, tj1 = by1 >> 3;  // floor
  const int nbr = bx1 >= bx0 ? ti1 - ti0 + 1 : 0, nbc = by1 >= by0 ? tj1 - tj0 + 1 : 0;
  const int nt = nbr * nbc;
  // the 5 x 5 tiles around the targets' bounding box (the end cells at the
  // quirk index sit pad cells up-left of the robot, the crop around it)
  const int tx_c = (min(px - pad - 1, px - s.ego) + max(px - pad + 1, px + s.ego)) >> 1;
  const int ty_c = (min(py - pad - 1, py - s.ego) + max(py - pad + 1, py + s.ego)) >> 1;
  const int rti0 = (tx_c >> 3) - 2, rtj0 = (ty_c >> 3) - 2;
  tried = nt + 25 + 40 <= kFastTiles;  // the box, the 5 x 5 tiles, their 40 rows
  if (!tried) return;
  // the thread's cached cells (cell, d): loads in flight with the tiles'
  constexpr int KC = (kDistK + NTH - 1) / NTH;
  int32_t pcw[KC], pcd[KC];
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const int k = tid + j * NTH;
    pcw[j] = k < ccnt ? cc[k] : 0;
    pcd[j] = k < ccnt ? cd[k] : 0;
  }
  for (int i = tid; i < nt + 25; i += NTH) {
    int ti, tj;
    if (i < nt) {
      const int r = i / nbc;
      ti = ti0 + r;
      tj = tj0 + (i - r * nbc);
    } else {
      const int r = (i - nt) / 5;
      ti = rti0 + r;
      tj = rtj0 + (i - nt - 5 * r);
    }
    uint64_t t = (ti >= 0 && ti < s.TR && tj >= 0 && tj < s.TC) ? free_t[tile_index(s.TCS, ti, tj)] : 0ull;
    const int rows = s.Wp - 8 * ti;  // the transform reads map rows < Wp only
    if (rows < 8) t &= rows > 0 ? low_mask(8 * rows) : 0ull;
    ft[i] = t;
  }
  __syncthreads();
  if (ts) DSTAMP(ts[0]);
  // the staged box (tile-aligned): rows [X0, X0 + 8 nbr), columns [Y0, Y0 + 8 nbc)
  const int X0 = 8 * ti0, Y0 = 8 * tj0, NR = 8 * nbr, NC = 8 * nbc;
  const bool rspan = span && nt > 0 && NR <= kSpan, cspan = span && nt > 0 && NC <= kSpan;
  if (rspan || cspan) {
    // row X: the first and last covered column (offsets from Y0; 0xFFFF: none);
    // column Y: the first and last covered row (offsets from X0)
    for (int i = tid; i < (rspan ? NR : 0) + (cspan ? NC : 0); i += NTH) {
      uint32_t lo = 0xFFFFu, hi = 0u;
      if (rspan && i < NR) {
        const uint64_t* trow = ft + (i >> 3) * nbc;
        const int sh = 8 * (i & 7);
        for (int j = 0; j < nbc; ++j) {
          const uint32_t b = (uint32_t)(trow[j] >> sh) & 0xFFu;
          if (b) {
            if (lo == 0xFFFFu) lo = 8 * j + __ffs(b) - 1;
            hi = 8 * j + 31 - __clz(b);
          }
        }
        span[i] = lo | (hi << 16);
      } else {
        const int y = i - (rspan ? NR : 0);
        const uint64_t m = 0x0101010101010101ull << (y & 7);
        for (int r = 0; r < nbr; ++r) {
          const uint64_t b = ft[r * nbc + (y >> 3)] & m;
          if (b) {
            if (lo == 0xFFFFu) lo = 8 * r + (__ffsll((unsigned long long)b) - 1) / 8;
            hi = 8 * r + (63 - __clzll((unsigned long long)b)) / 8;
          }
        }
        span[kSpan + y] = lo | (hi << 16);
      }
    }
    __syncthreads();
    // the extents' 1D transforms: along the row axis (q = box row)
    // tr[0][a] = min_q |a - q| + lo(q), tr[1][a] = min_q |a - q| - hi(q); the
    // same along the column axis in tr[2], tr[3] (kInf: no covered cell)
    int* tr = reinterpret_cast<int*>(span + 2 * kSpan);
    const int nr = rspan ? NR : 0, nc = cspan ? NC : 0;
    for (int i = tid; i < 2 * (nr + nc); i += NTH) {
      const bool rows = i < 2 * nr;
      const int k = rows ? i : i - 2 * nr, side = k & 1, a = k >> 1, n = rows ? nr : nc;
      const uint32_t* sp = rows ? span : span + kSpan;
      int best = kInf;
      for (int q = 0; q < n; ++q) {
        const uint32_t v = sp[q];
        if ((v & 0xFFFFu) == 0xFFFFu) continue;
        best = min(best, abs(a - q) + (side ? -(int)(v >> 16) : (int)(v & 0xFFFFu)));
      }
      tr[(rows ? 0 : 2 * kSpan) + side * kSpan + a] = best;
    }
    __syncthreads();
  }
  uint32_t mykey = 0;
#pragma unroll
  for (int j = 0; j < KC; ++j) {
    const int k = tid + j * NTH;
    if (k >= ccnt) break;
    const int32_t cw = pcw[j];
    const int cx = witness_x(cw), cy = witness_y(cw);
    int d = pcd[j];
    // only box tiles inside the cell's L1 ball of radius d can lower it (a
    // cell at least d from the box keeps its d): tile rows outward from the
    // cell's, each row's columns limited by the radius left (d shrinks as
    // covered cells turn up)
    const int bdist = max(0, max(bx0 - cx, cx - bx1)) + max(0, max(by0 - cy, cy - by1));
    const int gy = max(Y0 - cy, cy - (Y0 + NC - 1)), gx = max(X0 - cx, cx - (X0 + NR - 1));
    if (bdist < d && nt > 0 && ((rspan && gy > 0) || (cspan && gx > 0))) {
      // the cell is beside the box's column band (or row band): in every box
      // row the nearest covered cell is that row's first (last) covered
      // column, so d = min over rows |cx - X| + the column gap, one read of
      // the rows' 1D transform (a cell outside the row range: the nearest
      // row's value plus the distance to it)
      const bool byrow = rspan && gy > 0 && (!(cspan && gx > 0) || NR <= NC);
      const int a = byrow ? cx - X0 : cy - Y0, n = byrow ? NR : NC;  // the cell along the span axis
      const int o = byrow ? cy - Y0 : cx - X0;                          // and across it (outside [0, n'))
      const int* tr = reinterpret_cast<const int*>(span + 2 * kSpan) + (byrow ? 0 : 2 * kSpan);
      const int ac = min(max(a, 0), n - 1);
      const int v = o < 0 ? tr[ac] : tr[kSpan + ac];
      if (v < kInf / 2) d = min(d, abs(a - ac) + (o < 0 ? v - o : v + o));
    } else if (bdist < d && nt > 0) {
      const int ct = min(max(cx >> 3, ti0), ti1);  // the box tile row nearest the cell
      for (int dr = 0; dr <= nbr; ++dr) {
        bool any = false;
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          const int ti = sg ? ct + dr : ct - dr;
          if ((sg && dr == 0) || ti < ti0 || ti > ti1) continue;
          const int dx = max(0, max(8 * ti - cx, cx - (8 * ti + 7)));  // to the tile row band
          if (dx >= d) continue;
          any = true;
          const int rem = d - dx;
          const int c0 = max(tj0, (cy - rem) >> 3), c1 = min(tj1, (cy + rem) >> 3);
          const uint64_t* row = ft + (ti - ti0) * nbc - tj0;
          for (int tj = c0; tj <= c1; ++tj) d = tile_min_dist(row[tj], 8 * ti, 8 * tj, cx, cy, d);
        }
        if (!any && dr > 0) {  // both rows at this distance are out of the ball (or the box)
          const int dlo = 8 * (ct - dr) + 7 < cx ? cx - (8 * (ct - dr) + 7) : 0;
          const int dhi = 8 * (ct + dr) > cx ? 8 * (ct + dr) - cx : 0;
          if ((ct - dr < ti0 || dlo >= d) && (ct + dr > ti1 || dhi >= d)) break;
        }
      }
    }
    cdv[k] = d;
    mykey = max(mykey, ((uint32_t)d << 16) | (uint32_t)k);
  }
  if (ts) DSTAMP(ts[1]);
  mykey = wave_max_u32(mykey);
  if ((tid & 63) == 0) atomicMax(fkey, mykey);
  // target t, map coordinates: [0, 5) the end cells of the next step at the
  // quirk index (padded-grid x, y, no pad offset), then the crop
  auto target_cell = [&](int t, int& tx, int& ty) {
    if (t >= 5) {
      const int r = (t - 5) / E;
      tx = px - s.ego + r;
      ty = py - s.ego + (t - 5 - r * E);
    } else {
      tx = px + (t == 1 ? 1 : (t == 3 ? -1 : 0)) - pad;
      ty = py + (t == 2 ? 1 : (t == 4 ? -1 : 0)) - pad;
    }
  };
  // the 40 x 40 block as row words (bit c: column 8 rtj0 + c)
  uint64_t* brow = ft + nt + 25;
  for (int r = tid; r < 40; r += NTH) {
    uint64_t w = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) w |= ((ft[nt + (r >> 3) * 5 + c] >> (8 * (r & 7))) & 0xFFull) << (8 * c);
    brow[r] = w;
  }
  __syncthreads();
  // d of each target: rows outward from its own while the row distance
  // stays below the best d (a covered target, d = 0: one read); exact when
  // d <= b, the distance to the block's outside, else the map is not served
  for (int t = tid; t < T; t += NTH) {
    int tx, ty;
    target_cell(t, tx, ty);
    const int lx = tx - 8 * rti0, ly = ty - 8 * rtj0;
    const int b = min(min(lx, 39 - lx), min(ly, 39 - ly)) + 1;
    int d = b + 1;
    if (b > 0) {
      d = min(d, row_near(brow[lx], ly));
      for (int dr = 1; dr < d; ++dr) {
        const int up = lx - dr >= 0 ? row_near(brow[lx - dr], ly) : kInf;
        const int dn = lx + dr < 40 ? row_near(brow[lx + dr], ly) : kInf;
        d = min(d, dr + min(up, dn));
      }
    }
    if (d > b) *ffail = 1;
    else s_d[t] = d;
  }
  __syncthreads();
}

// a map the cache served: (M, witness), the cached d (exact again: an empty
// box), the PRE data and the obs crop.  NTH threads.
template <int NTH>
__device__ __forceinline__ void cache_serve(const State& s, int T, uint32_t ea, uint32_t fkey, int ccnt, int cM0,
                                            const uint16_t* cdv, const int* s_d, float* pre_out, float* dist_obs,
                                            uint32_t* count) {
  const int tid = opaque_tid(), E = s.E;
  const int M = (int)(fkey >> 16), kb = (int)(fkey & 0xFFFFu);
  const float Mf = (float)M;
  if (tid == 0) {
    if (count) atomicAdd(count + 3, 1u);  // maps the cache served (MC_FIELD_DIST_CACHED)
    reinterpret_cast<int2*>(s.dist_mw)[ea] = make_int2(M, s.dist_cc[(size_t)ea * kDistK + kb]);
    reinterpret_cast<int4*>(s.dist_ch + (size_t)ea * 8)[0] = make_int4(ccnt, cM0, 1 << 28, 1 << 28);
    reinterpret_cast<int2*>(s.dist_ch + (size_t)ea * 8)[2] = make_int2(-(1 << 28), -(1 << 28));
  }
  for (int k = tid; k < ccnt; k += NTH) s.dist_cd[(size_t)ea * kDistK + k] = cdv[k];
  float* dst = dist_obs + (size_t)ea * E * E;
  for (int t = 5 + tid; t < T; t += NTH) dst[t - 5] = dist_value((float)s_d[t], Mf);
  float* pd = pre_out + (size_t)ea * 8;
  if (tid == 0) pd[0] = Mf;
  if (tid < 5) pd[1 + tid] = (float)s_d[tid];
}

// Launch modes of dist_kernel_t:
//   0  every map (list == nullptr), or the listed maps, each whole in one
//      workgroup: the cache fast path, else the full transform
//   (1  the listed maps' cache fast path alone: dist_fast_kernel; a map it
//      cannot serve goes to the full list, `full`: [0] count, [2] the last
//      step's count; from [8] (map, theta0) pairs)
//   2  the full list, each map's strips split over S workgroups ("parts",
//      S from the list length: the few full transforms of a steady state
//      step are latency-bound in one workgroup): a part transforms its
//      strips and publishes its best key, strip maxima, target cells and
//      cache candidates (State::dist_g*); with S == 1 the one part
//      finalises the map as mode 0 does
//   3  the full list after mode 2 (S > 1): one workgroup per map merges the
//      parts' partials and finalises the map (the bitboard is staged only
//      for a second cache pass).  A launch boundary orders the parts'
//      stores before the merge: no per-map done counter, no device-scope
//      fences between the XCDs' L2s
constexpr int kSplitSlots = 512;  // workgroups resident at once (2 per CU)
#ifndef MC_MAX_PARTS  // build knob (A/B): parts per split map
#define MC_MAX_PARTS 8
#endif
constexpr int kMaxParts = MC_MAX_PARTS;
// the parts' candidate lists and counts are indexed by the map's full-list
// index: S > 1 parts only when at most kSplitSlots / 2 maps are on the list
// (State::dist_gcand was [B][N][4 kDistK], 2 GB at C5).  Round 6: one
// segment of kDistK per part ([kDistGSlots][kDistGParts][kDistK], 8 MB), so
// a part publishes its count with a plain store instead of taking its
// place with a returning atomic (MC_DIST_SEGS=0: one shared list of
// 4 kDistK, places by atomicAdd)
static_assert(kDistGSlots == kSplitSlots / 2, "State::dist_gcand's slots");
static_assert(kMaxParts <= kDistGParts, "State::dist_gcand's segments");
#ifndef MC_DIST_SEGS
#define MC_DIST_SEGS 1
#endif
constexpr bool kSegs = MC_DIST_SEGS != 0;
constexpr int kGCand = 4 * kDistK;  // (kSegs = 0) candidates a split map's parts may publish
#ifndef MC_DIST_FUSED  // build knob (A/B): 0 finalises split maps in a separate mode-3 launch
#define MC_DIST_FUSED 1
#endif
// the part of a split map that finishes last finalises it inside mode 2
// (`sc1` hand-off of the partials) instead of a mode-3 launch after it
constexpr bool kFused = MC_DIST_FUSED != 0;
#ifndef MC_DIST_XCD  // build knob (A/B): 1 keeps a split map's parts on one XCD
// (tried, round 5: the transform launch took 59.0 vs 54.3 us per C5 steady
// step with the parts spread over the XCDs, profiles/r5/xcd/)
#define MC_DIST_XCD 0
#endif
constexpr bool kXcdParts = MC_DIST_XCD != 0;
#ifndef MC_DIST_BALANCE  // build knob (A/B): 0 splits a map's strips evenly by count
#define MC_DIST_BALANCE 1
#endif
constexpr bool kBalance = MC_DIST_BALANCE != 0;
#ifndef MC_DIST_OPAQUE_TID  // build knob (A/B): 0 = round 5's item loop (VGPR spills at <17>)
#define MC_DIST_OPAQUE_TID 1
#endif
#ifndef MC_DIST_ACQREL  // build knob (A/B): 0 = round 5's relaxed arrival add (ordering by vmcnt + sc1 only)
#define MC_DIST_ACQREL 1
#endif
#ifndef MC_DIST_HO_SC1  // build knob (A/B): 0 = plain stores / loads for the hand-off (the acq_rel arrival orders them)
#define MC_DIST_HO_SC1 1
#endif
#ifndef MC_DIST_SKIP_IDLE  // build knob (A/B): 1 = idle parts skip staging (measured slower, round 6)
#define MC_DIST_SKIP_IDLE 0
#endif
// A part that the balanced split gives no running strip (fewer running
// strips than parts) stages nothing: it only arrives, and stages the map
// after all if it is the merger and the cache pass has to run.  Measured
// slower (C5 steady 142.5 vs 140.3 us, default window 153.7 vs 151.6 us,
// profiles/r6/hoab/): off
constexpr bool kSkipIdle = MC_DIST_SKIP_IDLE != 0;
#ifndef MC_DIST_STAGE1  // build knob (A/B): 0 keeps the two-pass staging (map rows, then extended rows)
#define MC_DIST_STAGE1 1
#endif
constexpr bool kStage1 = MC_DIST_STAGE1 != 0;
#ifndef MC_DIST_PARTLIST  // build knob (A/B): 1 = part lists (below); off: measured slower, round 6
#define MC_DIST_PARTLIST 0
#endif
// Part lists: a split map without a cache bound (theta0 = 0, e.g. every map
// early after a reset) -- each part collects its own cells with d >= its own
// maximum - kDistT (a superset of its cells with d >= M - kDistT, M >= that
// maximum) and publishes them like the one-pass candidates; a part whose
// maximum is below the best published key - kDistT holds no cache cell and
// skips it.  The merger then needs the serial cache pass only when a part
// that overflowed its list reaches M - kDistT (State::dist_govf).
// Measured slower (round 6, profiles/r6/dist/: C5 default window 162.5 vs
// 158.0 us per step, steady 150.8 vs 147.0): the parts' extra strip passes
// cost more than the merger's serial pass they save.  Kept as an A/B knob,
// parity-tested (tests/test_gpu_shapes.py, 8 envs: the mass reset splits
// every map with theta0 = 0).
constexpr bool kPartList = MC_DIST_PARTLIST != 0 && kOnePass;
// the split parts' hand-off words as agent-scope relaxed atomics (`sc1`),
// or, under the acq_rel arrival, plain stores and loads (no faster within
// the noise, profiles/r6/hoab/: kept sc1)
constexpr bool kHoSc1 = MC_DIST_HO_SC1 != 0 || MC_DIST_ACQREL == 0;

// The strips a full transform of map ea runs with the lower bound theta of
// its new max(d) (bit st; the rest are pruned, dist_kernel_t's strip loop):
// a strip runs if its last known maximum (State::dist_sm) reaches theta -
// kDistT or it holds a target cell.  Computed when the map goes to the full
// list (dist_fast_kernel), before any part of the next launch publishes new
// strip maxima: every part then splits the same running strips evenly.
__device__ uint64_t strip_run_mask(const State& s, int pad, uint32_t ea, int theta) {
  const int RY = s.Lp + 2 * pad, nst = (RY + kStrip - 1) / kStrip;
  const uint64_t all = nst >= 64 ? ~0ull : low_mask(nst);
  if (theta <= 0 || nst > kMaxTrack || !s.dist_sm) return all;
  const int2 pp = reinterpret_cast<const int2*>(s.pos)[ea];
  const int tv_lo = min(pp.y - 1, pp.y + pad - s.ego), tv_hi = max(pp.y + 1, pp.y + pad + s.ego);
  const uint32_t* smb = s.dist_sm + (size_t)ea * kMaxTrack;
  uint64_t m = 0;
  for (int st = 0; st < nst; ++st) {
    const int c0 = st * kStrip;
    if ((int)smb[st] >= theta - kDistT || (c0 + kStrip > tv_lo && c0 <= tv_hi)) m |= 1ull << st;
  }
  return m;
}

#ifndef MC_DIST_RELOAD  // build knob (A/B): 0 keeps one State for the whole kernel
#define MC_DIST_RELOAD 1
#endif
// The State re-read from the kernel arguments at the item's phase boundaries
// (as the env kernel's reload_state, mc_env_kernel.hip): the fields a phase
// uses are loaded there instead of living in SGPRs -- spilled to VGPR lanes,
// a VALU v_readlane per use -- across the item loop
struct DistIO {
  int pad, post;
  float* pre_out;   // [B][N][8] M, d of the 5 end cells
  float* dist_obs;  // [B][N][E][E] (POST)
  const uint32_t* list;
  uint32_t* count;
  int mode;
  uint32_t* full;
};
struct DistArgs {
  State s;
  DistIO io;
};
__device__ __forceinline__ void dist_reload(State& s, DistIO& io) {
  if constexpr (MC_DIST_RELOAD != 0) {
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();  // the DistArgs
    asm volatile("" : "+s"(kp));
    const DistArgs& A = *(const DistArgs*)kp;
    s = A.s;
    io = A.io;
  }
}

template <int kCL>
__global__ __launch_bounds__(kDtThreads, 4) void dist_kernel_t(DistArgs args) {
  State s = args.s;
  DistIO io = args.io;
  // the arguments as names for the current copy (dist_reload rewrites it)
  const int& pad = io.pad;
  const int& post = io.post;
  float* const& pre_out = io.pre_out;
  float* const& dist_obs = io.dist_obs;
  const uint32_t* const& list = io.list;
  uint32_t* const& count = io.count;
  const int& mode = io.mode;
  uint32_t* const& full = io.full;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_cov;
  __shared__ unsigned long long s_key;  // max over the map of (d, distance from the robot, cell)
  // top-cell cache (State::dist_ch): the fast path's best (d << 16 | index),
  // the strips' max(d), the cache pass's cell list
  __shared__ uint32_t s_fkey;
  __shared__ int s_ffail;
  __shared__ int s_ccount;
  __shared__ int s_kept;
  __shared__ uint32_t s_base;
  __shared__ int s_lb;
  __shared__ int s_smax[kMaxTrack];
  __shared__ int32_t s_ccell[kDistK];
  __shared__ uint16_t s_cdv[kDistK];  // d < 0xFFFF (the transform saturates there)
  const int tid = threadIdx.x;
  const int RX = s.Wp + 2 * pad, RY = s.Lp + 2 * pad, RW = (RY + 63) >> 6;
  const int E = s.E;
  const int T = post ? 5 + E * E : 5;
  const DtLds LL = dt_lds(RX, RY, s.MT, 5 + E * E);
  uint64_t* Cb = reinterpret_cast<uint64_t*>(smem);
  uint16_t* G = reinterpret_cast<uint16_t*>(smem + LL.cb);  // [kCh * kCL][kSP] (kStrip used)
  constexpr int RXP = kCh * kCL;                             // strip rows incl. padding
  int* s_d = reinterpret_cast<int*>(smem + LL.cb + LL.strip + LL.mins);
  const uint64_t last = (RY & 63) ? low_mask(RY & 63) : ~0ull;
  // every map (list == nullptr: one workgroup per (env, agent)), or the maps
  // of a device work list (a fixed grid strides over *count entries: the
  // count is uniform, so every wave reaches the end)
  const int nstrips_all = (RY + kStrip - 1) / kStrip;
  uint64_t tk = 0;  // (diagnostic) the workgroup's start
  DSTAMP(tk);
  const uint32_t nF = mode >= 2 ? __atomic_load_n(full, __ATOMIC_RELAXED) : 0u;
  const int S = mode >= 2 && nF > 0 ? max(1, min(min(nstrips_all, kMaxParts), (int)(kSplitSlots / nF))) : 1;
  // XCD-aware parts (mode 2, S > 1, a grid of whole XCD rounds): workgroup b
  // runs on XCD b % 8, so item it = 8 l + x is part l % S of map
  // 8 (l / S) + x -- every part of a map on one XCD, whose L2 then fetches
  // the map's tiles once for all of them (each part stages the whole map)
  const bool xcd = kXcdParts && mode == 2 && S > 1 && (gridDim.x & 7u) == 0u;
  ListView lv;
  lv.pre[kListShards] = 0;
  if (list && mode < 2) lv = list_view(s);
  const uint32_t n_items = mode == 2   ? (xcd ? ((nF + 7u) >> 3) * 8u * (uint32_t)S : nF * (uint32_t)S)
                           : mode == 3 ? (S > 1 ? nF : 0u)
                                       : (list ? lv.pre[kListShards] : (uint32_t)gridDim.x);
  const bool strided = mode >= 2 || list != nullptr;
  if (mode == 2 && blockIdx.x == 0 && tid == 0) {
    // mode 1 has drained the list: its counters for the diagnostics
    // (MC_FIELD_DIST_LISTED / _CACHED: every listed map was either served by
    // the cache or put on the full list -- no served-count atomic per
    // workgroup, all on one address) and empty for the next step's env
    // kernel (no per-workgroup done counters in modes 1 / 2; the env kernel
    // empties the full list)
    uint32_t nl = 0;
    for (int k = 0; k < kListShards; ++k) {
      nl += s.dist_shc[k * kShardStride];
      s.dist_shc[k * kShardStride] = 0;
    }
    count[2] = nl;
    count[4] = nl - nF;
    if (s.dist_tot) {  // MC_FIELD_DIST_TOTALS (one thread, stream-ordered)
      s.dist_tot[0] += nl;
      s.dist_tot[1] += nl - nF;
      s.dist_tot[2] += nF;
      s.dist_tot[3] += 1ull;
    }
    count[3] = 0;
  }
  for (uint32_t it = blockIdx.x; it < n_items; it += (strided ? gridDim.x : n_items)) {
    // the thread index, opaque per item: otherwise the compiler hoists every
    // per-thread address and lane mask of the item body out of the item loop
    // and keeps them live across it -- 24 VGPRs spilled to scratch (100 B per
    // lane, ~24 MB of scratch writes per C5 step) at <17>, none with this
#if MC_DIST_OPAQUE_TID
    const int tid = opaque_tid();
#else
    const int tid = threadIdx.x;
#endif
    dist_reload(s, io);
    // modes 2 / 3: the full-list entry (and mode 2's part)
    const uint32_t l = it >> 3;
    const uint32_t fi = mode == 2 ? (xcd ? (l / (uint32_t)S) * 8u + (it & 7u) : it / (uint32_t)S) : (mode == 3 ? it : 0u);
    const int part = mode == 2 ? (xcd ? (int)(l % (uint32_t)S) : (int)(it - fi * (uint32_t)S)) : 0;
    if (fi >= nF && mode == 2) continue;  // (xcd: this XCD's share ran out; uniform per workgroup)
    const uint32_t ea = mode >= 2 ? full[8 + 2 * fi] : (list ? list_entry(s, lv, list, it) : it);
    // the strips this workgroup transforms: a contiguous range, the ranges
    // splitting the map's running strips evenly (strip_run_mask; without a
    // mask, its strips)
    int st_lo = part * nstrips_all / S, st_hi = (part + 1) * nstrips_all / S;
    bool idle = false;  // no running strip in this part's range (kSkipIdle)
    if (kBalance && mode == 2 && S > 1 && s.dist_rmask) {
      const uint64_t rm = s.dist_rmask[ea];
      if (rm) {
        const int R = __popcll(rm);
        // the first strip of the part holding running strip of rank p R / S
        auto bound = [&](int p) -> int {
          if (p == 0) return 0;
          const int r = p * R / S;
          if (p >= S || r >= R) return nstrips_all;
          uint64_t m = rm;
          for (int k = 0; k < r; ++k) m &= m - 1ull;
          return __ffsll((unsigned long long)m) - 1;
        };
        st_lo = bound(part);
        st_hi = bound(part + 1);
        const uint64_t upto_hi = st_hi >= 64 ? ~0ull : low_mask(st_hi);
        const uint64_t upto_lo = st_lo >= 64 ? ~0ull : low_mask(st_lo);
        idle = kSkipIdle && (rm & upto_hi & ~upto_lo) == 0ull;
      }
    }
    uint64_t ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, dflags = 0, tsa = 0, tsb = 0;
    DSTAMP(ts0);
    const uint64_t* free_t = s.freem + (size_t)ea * s.MT;
    const int2 pp = reinterpret_cast<const int2*>(s.pos)[ea];
    const int px = pp.x, py = pp.y;

    // target t -> extended cell (u, v): [0, 5) the end cells of the next step
    // (quirk: distance_map[x, y] with the padded-grid (x, y), no pad offset),
    // [5, 5 + E*E) the crop (POST only)
    auto target = [&](int t, int& u, int& v) {
      if (t >= 5) {
        const int r = (t - 5) / E, c = (t - 5) - r * E;
        u = px + pad - s.ego + r;
        v = py + pad - s.ego + c;
      } else {
        u = px + (t == 1 ? 1 : (t == 3 ? -1 : 0));
        v = py + (t == 2 ? 1 : (t == 4 ? -1 : 0));
      }
    };
    for (int t = tid; t < T; t += kDtThreads) s_d[t] = -1;
    if (tid == 0) {
      s_key = 0;
      s_cov = 0;
      s_fkey = 0;
      s_ffail = 0;
      s_ccount = 0;
      s_kept = 0;
    }
    for (int i = tid; i < kMaxTrack; i += kDtThreads) s_smax[i] = 0;
    // every wave sees the scalars above before it reads one: s_fkey is read
    // for theta0 below even when no cache try (whose barriers would order it)
    // runs.  (Round 5's intermittent split/unsplit dist_obs mismatch at the
    // mass auto-reset of test_c5_unsplit_transform_is_identical: with no map
    // cached, waves of the unsplit path read the previous workgroup's s_fkey
    // out of LDS before thread 0 zeroed it, took its d as theta0, pruned
    // strips the other waves ran, and fell out of step at the strips'
    // barriers.)
    __syncthreads();
    // the map's top-cell cache (mc_internal.h State::dist_ch)
    int ccnt = -1, cM0 = 0, bx0 = 0, by0 = 0, bx1 = -1, by1 = -1;
    if (s.dist_ch) {
      const int4 h0 = reinterpret_cast<const int4*>(s.dist_ch + (size_t)ea * 8)[0];
      const int2 h1 = reinterpret_cast<const int2*>(s.dist_ch + (size_t)ea * 8)[2];
      ccnt = h0.x;
      cM0 = h0.y;
      bx0 = h0.z;
      by0 = h0.w;
      bx1 = h1.x;
      by1 = h1.y;
    }
    // ---- the top-cell cache fast path (cache_try) for a listed map
    bool fast = false, tried = false;
    if (mode < 2 && list != nullptr && ccnt > 0) {
      cache_try<kDtThreads>(s, pad, T, px, py, free_t, ccnt, bx0, by0, bx1, by1, reinterpret_cast<uint64_t*>(G),
                            s.dist_cc + (size_t)ea * kDistK, s.dist_cd + (size_t)ea * kDistK, s_cdv, s_d, &s_fkey,
                            &s_ffail, tried);
      fast = tried && s_ffail == 0 && (int)(s_fkey >> 16) >= cM0 - kDistT;
    }
    uint64_t tsf = 0;
    DSTAMP(tsf);
    // the exact current d of the cached cells (the fast path computed them
    // before it failed): a lower bound of the new max(d)
    // (a try that returned before staging -- box too large -- leaves none)
    const int theta0 = mode >= 2 ? (int)full[9 + 2 * fi] : (tried ? (int)(s_fkey >> 16) : 0);
    bool need_cb = true;  // the map's bitboard in LDS
    // ---- merge a split map's parts' partials: the best key, the raw target
    // d (in the output buffers), the strip maxima, the cache candidates.
    // Mode 3 (a launch after mode 2: plain loads), or the part of a fused
    // mode 2 that finished last (`sc1` loads of the parts' `sc1` stores)
    auto merge_parts = [&](bool sc1) {
      __syncthreads();  // the item's LDS scalars are initialised; every thread is past its own list
      if (tid == 0) s_ccount = 0;
      __syncthreads();
      // the parts' candidates: a one-pass list (with theta0), the part lists
      // (without), else none
      const bool lists = (kOnePass && theta0 > 0) || kPartList;
      // kSegs: part p's count and segment; pre[p] = the candidates before it
      uint32_t pre[kMaxParts + 1];
      pre[0] = 0u;
      bool over = false;
#pragma unroll
      for (int p = 0; p < kMaxParts; ++p) {
        const uint32_t c = (kSegs && lists && p < S) ? ld_ho(s.dist_gcnt + (size_t)fi * kDistGParts + p, sc1) : 0u;
        over |= c > (uint32_t)kDistK;
        pre[p + 1] = pre[p] + (c > (uint32_t)kDistK ? 0u : c);
      }
      const uint32_t total = kSegs ? pre[kMaxParts] : (lists ? ld_ho(s.dist_gcnt + fi, sc1) : 0u);
      const unsigned long long gk = ld_ho(s.dist_gkey + ea, sc1);
      const int thr = (int)(gk >> 48) - kDistT;  // the candidates that are cache cells
      // a part list that overflowed and may hold cache cells: the serial pass
      const uint32_t ovf = (kPartList && theta0 == 0) ? ld_ho(s.dist_govf + fi, sc1) : 0u;
      for (int t = tid; t < T; t += kDtThreads)
        s_d[t] = (int)(t < 5 ? ld_ho(pre_out + (size_t)ea * 8 + 1 + t, sc1)
                             : ld_ho(dist_obs + (size_t)ea * E * E + (t - 5), sc1));
      for (int st = tid; st < min(nstrips_all, kMaxTrack); st += kDtThreads)
        s_smax[st] = (int)ld_ho(s.dist_sm + (size_t)ea * kMaxTrack + st, sc1);
      if (gk != 0 && (kSegs ? !over : total <= (uint32_t)kGCand))
        for (int k = tid; k < (int)total; k += kDtThreads) {
          size_t at = (size_t)fi * kGCand + k;
          if constexpr (kSegs) {  // segment p holds candidates pre[p] .. pre[p + 1] - 1
            uint32_t base = 0u;
            int p = 0;
#pragma unroll
            for (int q = 1; q < kMaxParts; ++q)
              if ((uint32_t)k >= pre[q]) {
                p = q;
                base = pre[q];
              }
            at = ((size_t)fi * kDistGParts + p) * kDistK + ((uint32_t)k - base);
          }
          const int2 c = ld_ho(s.dist_gcand + at, sc1);
          if (c.y >= thr) {
            const int j = atomicAdd(&s_ccount, 1);
            if (j < kDistK) {
              s_ccell[j] = c.x;
              s_cdv[j] = (uint16_t)c.y;
            }
          }
        }
      __syncthreads();
      if (tid == 0) {
        s_key = gk;
        s_cov = gk != 0;  // a covered map's key is nonzero (its far or cell field)
        if (kSegs ? over : total > (uint32_t)kGCand) s_ccount = kDistK + 1;  // overflowed: the second pass
        if (ovf > 0u && (int)ovf - 1 >= thr) s_ccount = kDistK + 1;
        s.dist_gkey[ea] = 0;  // zero for the map's next split transform
        if (!kSegs) s.dist_gcnt[fi] = 0;
        if (kPartList) s.dist_govf[fi] = 0;
      }
      if (kSegs && tid < S) s.dist_gcnt[(size_t)fi * kDistGParts + tid] = 0;
      __syncthreads();
    };
    if (mode == 3) {
      merge_parts(false);
      need_cb = s_cov && !(((kOnePass && theta0 > 0) || kPartList) && s_ccount <= kDistK);  // the second pass
    }
    // the map's row bitboard (Cb) in LDS
    auto stage_cb = [&]() {
      if (kStage1 && pad <= 16) {
        // one pass: a thread takes extended word w of one tile row (8 map
        // rows), loads the 8 tiles of map word w and the tile pair 8w-2,
        // 8w-1 (the last pad <= 16 columns of map word w-1, shifted in from
        // the left), transposes their bytes with v_perm into the 8 rows'
        // words and writes them, shifted right by pad, straight into the
        // extended rows pad + 8 ti + r of Cb.  The pad rows above and below
        // the map are zeroed.  (Round 5's two passes staged map rows in the
        // strip area first and extended them in a second LDS pass: ~6.8k of
        // a part's ~16k staging cycles at the C5 steady state,
        // profiles/r6/stamps/dist_steady.txt.)
        int any = 0;
        const int nq = s.TR * RW;
        for (int q0 = tid; q0 < nq; q0 += 2 * kDtThreads) {
          uint32_t lo[2][8], hi[2][8], plo[2][2], phi[2][2];  // word w's tiles; tiles 8w-2, 8w-1
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int q = q0 + k * kDtThreads;
            const int ti = q / RW, w = q - ti * RW;
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              const int tj = 8 * w + j;
              uint4 t = make_uint4(0u, 0u, 0u, 0u);
              if (q < nq && tj < s.TC) t = *reinterpret_cast<const uint4*>(free_t + tile_index(s.TCS, ti, tj));
              if (tj + 1 >= s.TC) t.z = t.w = 0u;
              lo[k][j] = t.x;
              hi[k][j] = t.y;
              lo[k][j + 1] = t.z;
              hi[k][j + 1] = t.w;
            }
            const int tp = 8 * w - 2;  // even: one 16-byte load (both tiles < TC when w <= RWm)
            uint4 t = make_uint4(0u, 0u, 0u, 0u);
            if (q < nq && pad > 0 && w > 0 && tp < s.TC) t = *reinterpret_cast<const uint4*>(free_t + tile_index(s.TCS, ti, tp));
            if (tp + 1 >= s.TC) t.z = t.w = 0u;
            plo[k][0] = t.x;
            phi[k][0] = t.y;
            plo[k][1] = t.z;
            phi[k][1] = t.w;
          }
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int q = q0 + k * kDtThreads;
            if (q >= nq) break;
            const int ti = q / RW, w = q - ti * RW;
            const int nr = min(8, s.Wp - 8 * ti);
            const uint64_t wm = (w == RW - 1) ? last : ~0ull;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              if (r >= nr) break;
              const uint32_t* src = r < 4 ? lo[k] : hi[k];
              const uint32_t* psrc = r < 4 ? plo[k] : phi[k];
              const uint32_t b = (uint32_t)(r & 3);
              // byte b of src[j]: pairs (j, j + 1) -> bytes 0, 1 of a dword,
              // then two such pairs -> 4 bytes
              const uint32_t sel2 = b | ((4u + b) << 8) | 0x0C0C0000u;
              const uint32_t p01 = __builtin_amdgcn_perm(src[1], src[0], sel2);
              const uint32_t p23 = __builtin_amdgcn_perm(src[3], src[2], sel2);
              const uint32_t p45 = __builtin_amdgcn_perm(src[5], src[4], sel2);
              const uint32_t p67 = __builtin_amdgcn_perm(src[7], src[6], sel2);
              const uint32_t wlo = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
              const uint32_t whi = __builtin_amdgcn_perm(p67, p45, 0x05040100u);
              const uint64_t cur = (uint64_t)wlo | ((uint64_t)whi << 32);
              // bits 48..63 of map word w - 1 (tiles 8w-2, 8w-1) as 16 bits
              const uint32_t prev16 = __builtin_amdgcn_perm(psrc[1], psrc[0], sel2);
              const uint64_t c = (pad > 0 ? ((cur << pad) | (uint64_t)(prev16 >> (16 - pad))) : cur) & wm;
              Cb[(size_t)(pad + 8 * ti + r) * RW + w] = c;
              any |= c != 0ull;
            }
          }
        }
        // the extended rows outside the map
        const int below = RX - pad - s.Wp;
        for (int i = tid; i < (pad + below) * RW; i += kDtThreads) {
          const int row = i / RW;
          Cb[(size_t)(row < pad ? row : row + s.Wp) * RW + (i - row * RW)] = 0ull;
        }
        DSTAMP(tsa);
        DSTAMP(tsb);
        if (any) s_cov = 1;
      } else {
        // the agent's tiles as map rows in the strip area (free until the
        // strips start): a thread takes 8 tiles of one tile row (one 64-column
        // word of 8 map rows), loads them, and transposes their bytes with
        // v_perm -- byte j of row word r = byte r of tile j -- into 8 word
        // stores (was 64 byte stores per 8 tiles).  Tiles past the last tile
        // column load as 0.  Then the extended rows: map columns shifted
        // right by pad (a funnel shift of two words)
        uint8_t* crow = reinterpret_cast<uint8_t*>(G);
        uint64_t* crw = reinterpret_cast<uint64_t*>(G);
        const int RWm = (s.TC + 7) >> 3;  // u64 words per map row
        const int nq = s.TR * RWm;
        // two items per thread per round, every load of both issued first
        // (a 514-row map has 585 items: one round of load latency, not two)
        for (int q0 = tid; q0 < nq; q0 += 2 * kDtThreads) {
          uint32_t lo[2][8], hi[2][8];  // tile j's dwords (rows 0-3, rows 4-7)
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int q = q0 + k * kDtThreads;
            const int ti = q / RWm, w = q - ti * RWm;
            // tiles (ti, tj), (ti, tj + 1) of an even tj are adjacent in the
            // block layout: one 16-byte load per pair (the block's padding
            // columns exist; a tile past the last column reads as 0)
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
              const int tj = 8 * w + j;
              uint4 t = make_uint4(0u, 0u, 0u, 0u);
              if (q < nq && tj < s.TC) t = *reinterpret_cast<const uint4*>(free_t + tile_index(s.TCS, ti, tj));
              if (tj + 1 >= s.TC) t.z = t.w = 0u;
              lo[k][j] = t.x;
              hi[k][j] = t.y;
              lo[k][j + 1] = t.z;
              hi[k][j + 1] = t.w;
            }
          }
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int q = q0 + k * kDtThreads;
            if (q >= nq) break;
            const int ti = q / RWm, w = q - ti * RWm;
            const int nr = min(8, s.Wp - 8 * ti);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              if (r >= nr) break;
              const uint32_t* src = r < 4 ? lo[k] : hi[k];
              const uint32_t b = (uint32_t)(r & 3);
              // byte b of src[j]: pairs (j, j + 1) -> bytes 0, 1 of a dword,
              // then two such pairs -> 4 bytes
              const uint32_t sel2 = b | ((4u + b) << 8) | 0x0C0C0000u;
              const uint32_t p01 = __builtin_amdgcn_perm(src[1], src[0], sel2);
              const uint32_t p23 = __builtin_amdgcn_perm(src[3], src[2], sel2);
              const uint32_t p45 = __builtin_amdgcn_perm(src[5], src[4], sel2);
              const uint32_t p67 = __builtin_amdgcn_perm(src[7], src[6], sel2);
              const uint32_t wlo = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
              const uint32_t whi = __builtin_amdgcn_perm(p67, p45, 0x05040100u);
              crw[(size_t)(8 * ti + r) * RWm + w] = (uint64_t)wlo | ((uint64_t)whi << 32);
            }
          }
        }
        DSTAMP(tsa);
        __syncthreads();
        DSTAMP(tsb);
        const uint64_t* cw = reinterpret_cast<const uint64_t*>(crow);
        int any = 0;
        // a (row, word) item per thread and round (RX rows of RW words: 532
        // rows would leave 20 threads two whole rows)
        const int du = kDtThreads / RW, dw = kDtThreads - du * RW;
        int u = tid / RW, w = tid - u * RW;
        for (int idx = tid; idx < RX * RW; idx += kDtThreads) {
          const int X = u - pad;
          uint64_t c = 0;
          if (X >= 0 && X < s.Wp) {  // map columns [64 w - pad, 64 w - pad + 64)
            const int off = 64 * w - pad, ws = off >> 6, sh = off & 63;  // floor
            const uint64_t a0 = (ws >= 0 && ws < RWm) ? cw[X * RWm + ws] : 0ull;
            const uint64_t a1 = (ws + 1 >= 0 && ws + 1 < RWm) ? cw[X * RWm + ws + 1] : 0ull;
            c = sh ? ((a0 >> sh) | (a1 << (64 - sh))) : a0;
          }
          c &= (w == RW - 1) ? last : ~0ull;
          Cb[idx] = c;
          any |= c != 0;
          w += dw;
          u += du;
          if (w >= RW) {
            w -= RW;
            ++u;
          }
        }
        if (any) s_cov = 1;
      }
      __syncthreads();
    };
    if (!fast && need_cb && !idle) {
      if (mode != 3)  // (mode 3 holds the parts' targets)
        for (int t = tid; t < T; t += kDtThreads) s_d[t] = -1;
      stage_cb();
    }
    bool cov = fast || s_cov != 0;
    DSTAMP(ts1);
    dist_reload(s, io);

    // row-pass registers: a thread owns rows tid and tid + kDtThreads
    int lastL[2] = {-kInf, -kInf};  // last covered column left of the strip
    int nrw[2] = {-1, -1};          // next non-empty word after the current one (-1: not scanned)
    const int chunk = tid & (kCh - 1), pair = tid / kCh;
    const int u0c = chunk * kCL;
    // the chunk's rows inside the grid (only the last chunk has padding)
    const int nin = max(min(RX - u0c, kCL), 0);
    const uint32_t rowmask = nin >= 32 ? ~0u : ((1u << nin) - 1u);
    // best (d << 16 | u) of this thread's cells (ties: the largest u)
    uint32_t bestkey = 0;
    int bestv = -1;
    // bounding box of the target cells (extended coordinates): the column
    // chunks inside it keep their d in the strip for the target reads
    const int tu_lo = min(px - 1, px + pad - s.ego), tu_hi = max(px + 1, px + pad + s.ego);
    const int tv_lo = min(py - 1, py + pad - s.ego), tv_hi = max(py + 1, py + pad + s.ego);
    // one strip: thr < 0 -- the transform pass (keys, targets, strip maxima;
    // with cthr >= 0 also the cells with d >= cthr into the LDS list);
    // thr >= 0 -- the cache pass (cells with d >= thr into the LDS list)
    auto strip = [&](int st, int thr, int cthr) {
      const int c0 = st * kStrip, w = c0 >> 6, h = (c0 >> 5) & 1;
      // ---- row pass: g of the strip's 32 cells of row u, as 16 u16 pairs
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int u = tid + q * kDtThreads;
        if (u >= RXP) continue;
        uint2* grow = reinterpret_cast<uint2*>(G + u * kSP);
        if (u >= RX) {  // padding rows: no covered cell
#pragma unroll
          for (int k = 0; k < 8; ++k) grow[k] = make_uint2(~0u, ~0u);
          continue;
        }
        const uint64_t cw = Cb[u * RW + w];
        const uint32_t sb = (uint32_t)(cw >> (32 * h));
        // first covered column right of the strip
        int firstR = kInf;
        const uint32_t hb = h ? 0u : (uint32_t)(cw >> 32);
        if (hb) {
          firstR = c0 + 32 + __ffs(hb) - 1;
        } else {
          if (nrw[q] <= w) {  // scan for the next non-empty word (amortised O(RW) per row)
            int k = w + 1;
            while (k < RW && Cb[u * RW + k] == 0) ++k;
            nrw[q] = k;
          }
          if (nrw[q] < RW) firstR = 64 * nrw[q] + __ffsll((unsigned long long)Cb[u * RW + nrw[q]]) - 1;
        }
        const int lc = lastL[q];
        // (each 4-column uint2 is stored as soon as it is computed: the
        // strip's 16 packed pairs never all live in registers at once)
        if (sb == 0u) {
          // no covered cell in the strip: g(j) = min(A + j, B - j), two cells per packed op
          const uint32_t A = (uint32_t)min(c0 - lc, 0xFFFF - kStrip);
          const uint32_t Bd = (uint32_t)min(firstR - c0, 0xFFFF);  // >= 32
          const u16x2 Ap = {(uint16_t)A, (uint16_t)A}, Bp = {(uint16_t)Bd, (uint16_t)Bd};
#pragma unroll
          for (int k = 0; k < kStrip / 4; ++k) {
            const u16x2 c0j = {(uint16_t)(4 * k), (uint16_t)(4 * k + 1)};
            const u16x2 c1j = {(uint16_t)(4 * k + 2), (uint16_t)(4 * k + 3)};
            const u16x2 g0 = __builtin_elementwise_min(Ap + c0j, Bp - c0j);
            const u16x2 g1 = __builtin_elementwise_min(Ap + c1j, Bp - c1j);
            grow[k] = make_uint2(__builtin_bit_cast(uint32_t, g0), __builtin_bit_cast(uint32_t, g1));
          }
        } else if (sb == ~0u) {
#pragma unroll
          for (int k = 0; k < kStrip / 4; ++k) grow[k] = make_uint2(0u, 0u);
        } else {
          // g of each cell: nearest covered column at or left of it / at or
          // right of it (inside the strip by bit scans, else the carries)
#pragma unroll
          for (int j4 = 0; j4 < kStrip; j4 += 4) {
            uint32_t pp[2];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const int j = j4 + 2 * h2;
              int gg[2];
#pragma unroll
              for (int k = 0; k < 2; ++k) {
                const uint32_t le = sb & (0xFFFFFFFFu >> (31 - (j + k)));
                const uint32_t ge = sb & (0xFFFFFFFFu << (j + k));
                const int left = le ? c0 + 31 - __clz(le) : lc;
                const int right = ge ? c0 + __ffs(ge) - 1 : firstR;
                gg[k] = min(min(c0 + j + k - left, right - (c0 + j + k)), 0xFFFF);
              }
              pp[h2] = (uint32_t)gg[0] | ((uint32_t)gg[1] << 16);
            }
            grow[j4 >> 2] = make_uint2(pp[0], pp[1]);
          }
          lastL[q] = c0 + 31 - __clz(sb);
        }
        if (sb == ~0u) lastL[q] = c0 + 31;
      }
      __syncthreads();
      // ---- column pass: column pair p (columns c0 + 2p, c0 + 2p + 1 as the
      // low / high u16 halves of one packed register; saturating u16 pairs,
      // 0xFFFF = no covered cell) over chunk c of kCL rows.  u0 is made opaque
      // per strip: the compiler would otherwise hoist kCL loop-invariant row
      // values out of the strip loop (and spill them)
      int u0 = u0c;
      asm volatile("" : "+v"(u0));
      const uint32_t* g32 = reinterpret_cast<const uint32_t*>(G) + u0 * (kSP / 2) + pair;
      u16x2 tp[kCL], sd[kCL];  // g + K - u (then d), g + u (then the "down" distance)
      u16x2 pm = kNone2, sm = kNone2;
#pragma unroll
      for (int i = 0; i < kCL; ++i) {
        const u16x2 g = __builtin_bit_cast(u16x2, g32[i * (kSP / 2)]);
        const u16x2 uu = splat2(u0 + i);
        tp[i] = __builtin_elementwise_sub_sat(__builtin_elementwise_add_sat(g, kRowOff2), uu);
        sd[i] = __builtin_elementwise_add_sat(g, uu);
        pm = __builtin_elementwise_min(pm, tp[i]);
        sm = __builtin_elementwise_min(sm, sd[i]);
      }
      __syncthreads();  // every G read of the strip is done: the next row pass may write
      // minima over the pair's chunks before / after this one (its 32 chunks
      // are the lanes of one half wave)
      u16x2 run, sfx;
      if constexpr (kCh == 64) {
        run = excl_prefix_min64(pm);
        sfx = excl_suffix_min64(sm);
      } else {
        run = excl_prefix_min32(pm);
        sfx = excl_suffix_min32(sm);
      }
      // suffix scan: the "down" distance min_{u'>=u} g(u') + u' - u
#pragma unroll
      for (int i = kCL - 1; i >= 0; --i) {
        sfx = __builtin_elementwise_min(sfx, sd[i]);
        sd[i] = __builtin_elementwise_sub_sat(sfx, splat2(u0 + i));
      }
      // prefix scan, d = min(up, down), the best (d << 16 | u) of each column
      // over the chunk's grid rows (the last chunk's padding rows count 0)
      uint32_t klo = 0, khi = 0;
#pragma unroll
      for (int i = 0; i < kCL; ++i) {
        const u16x2 uu = splat2(u0 + i);
        run = __builtin_elementwise_min(run, tp[i]);
        const u16x2 up = __builtin_elementwise_sub_sat(__builtin_elementwise_add_sat(run, uu), kRowOff2);
        const uint32_t d = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(up, sd[i])) &
                           (uint32_t)__builtin_amdgcn_sbfe((int)rowmask, i, 1);
        tp[i] = __builtin_bit_cast(u16x2, d);
        klo = max(klo, (d << 16) | (uint32_t)(u0 + i));
        khi = max(khi, (d & 0xFFFF0000u) | (uint32_t)(u0 + i));
      }
      const int v = c0 + 2 * pair;
      const int collect = thr >= 0 ? thr : cthr;
      // cells with d >= collect into the LDS list; an overflowed list (count
      // > kDistK) is dropped whole: no more atomics
      if (collect >= 0 && *reinterpret_cast<volatile int*>(&s_ccount) <= kDistK) {
#pragma unroll
        for (int i = 0; i < kCL; ++i) {
          const uint32_t d = __builtin_bit_cast(uint32_t, tp[i]);
          const int dl = (int)(d & 0xFFFFu), dh = (int)(d >> 16);
          const bool row_in = (rowmask >> i) & 1u;
          if (row_in && v < RY && dl >= collect) {
            const int idx = atomicAdd(&s_ccount, 1);
            if (idx < kDistK) {
              s_ccell[idx] = pack_witness(u0 + i - pad, v - pad);
              s_cdv[idx] = dl;
            }
          }
          if (row_in && v + 1 < RY && dh >= collect) {
            const int idx = atomicAdd(&s_ccount, 1);
            if (idx < kDistK) {
              s_ccell[idx] = pack_witness(u0 + i - pad, v + 1 - pad);
              s_cdv[idx] = dh;
            }
          }
        }
      }
      if (thr >= 0) return;
      if (v < RY && klo > bestkey) {
        bestkey = klo;
        bestv = v;
      }
      if (v + 1 < RY && khi > bestkey) {
        bestkey = khi;
        bestv = v + 1;
      }
      if (s.dist_ch && st < kMaxTrack) {  // the strip's max(d), for the cache pass
        const uint32_t sm2 = wave_max_u32(max(v < RY ? klo >> 16 : 0u, v + 1 < RY ? khi >> 16 : 0u));
        if ((tid & 63) == 0) atomicMax(&s_smax[st], (int)sm2);
      }
      const bool keep = v + 1 >= tv_lo && v <= tv_hi && u0 + kCL > tu_lo && u0 <= tu_hi;
      if (keep) {  // the target cells of this chunk's columns, from registers
        for (int t = 0; t < T; ++t) {
          int tu, tv;
          target(t, tu, tv);
          if ((tv == v || tv == v + 1) && tu >= u0 && tu < u0 + kCL && tu < RX) {
            uint32_t val = 0;
#pragma unroll
            for (int i = 0; i < kCL; ++i) val = (u0 + i == tu) ? __builtin_bit_cast(uint32_t, tp[i]) : val;
            s_d[t] = (int)(tv == v ? (val & 0xFFFFu) : (val >> 16));
          }
        }
      }
    };
    const int nstrips = (cov && !fast && mode != 3) ? nstrips_all : 0;
    // The cache's cells in the same pass: every cell with d >= M - kDistT
    // (M = the new max, known only at the end) has d >= any lower bound of
    // M, less kDistT.  Bounds: theta0 and the strips' maxima so far (s_smax
    // two strips back: past two barriers).  The list then holds a superset,
    // filtered at the end; without a bound (no cache tried) or on overflow, a
    // second pass over the strips collects them.
    // Strip pruning (with theta0): a strip whose max(d) at the last full
    // transform (State::dist_sm, an upper bound now: d only decreases) is
    // below theta0 - kDistT holds neither the new max, nor a witness, nor a
    // cache cell; only its rows' last covered column is carried.  The
    // strips of the target cells always run.  (Tried: strips in descending
    // order of their bound with the exact maxima so far as the bound, a
    // barrier per strip: slower, 263 vs 242 us per step at C5.)
    const bool prune = theta0 > 0 && nstrips_all <= kMaxTrack;
    const uint32_t* smb = s.dist_ch ? s.dist_sm + (size_t)ea * kMaxTrack : nullptr;
    int runmax = 0;
    uint64_t ran = 0;  // strips transformed (their s_smax are exact maxima)
    const int s_from = nstrips > 0 ? st_lo : 0, s_to = nstrips > 0 ? st_hi : 0;
    // a part's first strip st0: each row's last covered column left of it
    auto carry_in = [&](int st0) {
      lastL[0] = lastL[1] = -kInf;
      nrw[0] = nrw[1] = -1;
      if (st0 == 0) return;
      const int c0 = st0 * kStrip, w = c0 >> 6;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int u = tid + q * kDtThreads;
        if (u >= RX) continue;
        uint64_t m = (c0 & 63) ? Cb[u * RW + w] & low_mask(c0 & 63) : 0ull;
        int k = w;
        while (!m && k > 0) m = Cb[u * RW + --k];
        if (m) lastL[q] = 64 * k + 63 - __clzll((unsigned long long)m);
      }
    };
    // a strip the pass skips: only its rows' last covered column is carried
    auto carry_over = [&](int st) {
      const int c0 = st * kStrip, w = c0 >> 6, h = (c0 >> 5) & 1;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int u = tid + q * kDtThreads;
        if (u >= RX) continue;
        const uint32_t sb = (uint32_t)(Cb[u * RW + w] >> (32 * h));
        if (sb) lastL[q] = c0 + 31 - __clz(sb);
      }
    };
    if (s_from > 0 && s_from < s_to) carry_in(s_from);
    for (int st = s_from; st < s_to; ++st) {
      if (st - 2 >= s_from && st - 2 < kMaxTrack && ((ran >> (st - 2)) & 1ull)) runmax = max(runmax, s_smax[st - 2]);
      if (prune) {
        const int c0 = st * kStrip, bound = smb[st];
        if (bound < theta0 - kDistT && !(c0 + kStrip > tv_lo && c0 <= tv_hi)) {
          if (tid == 0) s_smax[st] = bound;
          carry_over(st);
          continue;
        }
      }
      ran |= 1ull << (st < 64 ? st : 63);
      // (a bound below kDistT: every cell is a candidate, d >= 0 -- the list
      // then overflows and the cache pass runs; a negative threshold would
      // collect nothing and leave the list short)
      strip(st, -1, (kOnePass && theta0 > 0) ? max(max(theta0, runmax) - kDistT, 0) : -1);
    }
    DSTAMP(ts2);
    dist_reload(s, io);
    const int vmax = bestv >= 0 ? (int)(bestkey >> 16) : -1;
    const int ubest = (int)(bestkey & 0xFFFF), vbest = bestv;
    // witness: of the maxima, the one farthest from the robot (new coverage
    // comes from around the robot, so it keeps M valid longest)
    if (!fast && cov && vmax >= 0) {
      const int far = abs(ubest - (px + pad)) + abs(vbest - (py + pad));
      // 16 bits per field: d, far, u, v are all < 65535 (mc_create bounds
      // width + length + 4 pad), so wide grids keep an exact witness
      atomicMax(&s_key, ((unsigned long long)vmax << 48) | ((unsigned long long)far << 32) |
                            ((unsigned long long)ubest << 16) | (unsigned long long)vbest);
    }
    __syncthreads();
    bool merged = false;  // this part finalises its split map (fused mode 2)
    if (mode == 2 && S > 1) {
      // ---- a part: publish the best key, the targets it holds (raw d in
      // the output buffers), its strips' maxima and its cache candidates;
      // the part that finishes last (fused) or mode 3 finalises the map
      if (tid == 0 && s_key) atomicMax(s.dist_gkey + ea, s_key);
      for (int t = tid; t < T; t += kDtThreads)
        if (s_d[t] >= 0) {
          if (t < 5) st_ho(pre_out + (size_t)ea * 8 + 1 + t, (float)s_d[t], kFused && kHoSc1);
          else st_ho(dist_obs + (size_t)ea * E * E + (t - 5), (float)s_d[t], kFused && kHoSc1);
        }
      for (int st = st_lo + tid; st < min(st_hi, kMaxTrack); st += kDtThreads)
        if ((ran >> st) & 1ull) st_ho(s.dist_sm + (size_t)ea * kMaxTrack + st, (uint32_t)min(s_smax[st], 0xFFFF), kFused && kHoSc1);
      bool part_list = false;  // this part collected its own candidates (theta0 = 0)
      if (kPartList && theta0 == 0 && s.dist_ch) {
        // the part's own maximum and the best key the parts published so far
        // (a lower bound of M): below it by more than kDistT, no cache cell
        if (tid == 0) {
          const unsigned long long g = __hip_atomic_load((g_u64*)(s.dist_gkey + ea), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
          s_lb = (int)(max(g, (unsigned long long)s_key) >> 48);
          s_ccount = 0;
        }
        __syncthreads();
        const int pm = s_key ? (int)(s_key >> 48) : -1;
        if (pm >= 0 && pm >= s_lb - kDistT) {
          part_list = true;
          const int thr = max(pm - kDistT, 0);
          carry_in(st_lo);
          for (int st = st_lo; st < st_hi; ++st) {
            if (st >= kMaxTrack || s_smax[st] >= thr) {
              strip(st, thr, -1);
              __syncthreads();
              if (s_ccount > kDistK) break;  // overflowed: the merger's pass if it matters
            } else {
              carry_over(st);
            }
          }
          __syncthreads();
          if (tid == 0 && s_ccount > kDistK) atomicMax(s.dist_govf + fi, (uint32_t)pm + 1u);
        }
      }
      if ((kOnePass && theta0 > 0) || part_list) {
        const int n = s_ccount;
        if (n > 0 && (n <= kDistK || theta0 > 0)) {
          if constexpr (kSegs) {  // this part's segment and count (kDistK + 1: overflowed)
            const size_t sg = (size_t)fi * kDistGParts + part;
            if (tid == 0) st_ho(s.dist_gcnt + sg, (uint32_t)min(n, kDistK + 1), kFused && kHoSc1);
            if (n <= kDistK)
              for (int k = tid; k < n; k += kDtThreads)
                st_ho(s.dist_gcand + sg * kDistK + k, make_int2(s_ccell[k], s_cdv[k]), kFused && kHoSc1);
          } else {
            if (tid == 0) s_base = atomicAdd(s.dist_gcnt + fi, (uint32_t)(n <= kDistK ? n : kGCand + 1));
            __syncthreads();
            const uint32_t base = s_base;
            if (n <= kDistK)
              for (int k = tid; k < n; k += kDtThreads)
                if (base + k < (uint32_t)kGCand)
                  st_ho(s.dist_gcand + (size_t)fi * kGCand + base + k, make_int2(s_ccell[k], s_cdv[k]), kFused && kHoSc1);
          }
        }
      }
      if constexpr (kFused) {
        // every storing wave's stores done, then one arrival per part: an
        // agent-scope acq_rel add (release: the part's published words are
        // visible at agent scope before the count moves -- buffer_wbl2 of the
        // XCD's L2 after the waves' stores have completed; acquire: the
        // merger's loads after it miss its L1 / L2, buffer_inv).  The last
        // to arrive merges (its other waves read after the barrier)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
          s_base = MC_DIST_ACQREL ? __hip_atomic_fetch_add(s.dist_pcnt + ea, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                                  : atomicAdd(s.dist_pcnt + ea, 1u);
        __syncthreads();
        merged = s_base == (uint32_t)S - 1u;
        if (merged && tid == 0)  // zero for the map's next split transform
          __hip_atomic_store(s.dist_pcnt + ea, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (merged) {
        // the map's bitboard is staged here (every part stages it): a second
        // cache pass, if the parts' lists overflowed, needs no restaging
        merge_parts(kHoSc1);
        cov = s_cov != 0;  // the map's, from the parts' keys (an idle merger staged nothing)
      }
#ifdef MC_DIST_STAMPS
      {  // a part (flag bit 52): stage, strips, publish (mode 3 leaves these)
        uint64_t tp = 0;
        DSTAMP(tp);
        if (tid == 0 && s.stamps && ea < (uint32_t)s.B * 16u) {
          auto f16 = [](uint64_t a, uint64_t b) -> uint64_t {
            const uint64_t d = (b - a) >> 4;
            return d < 0xFFFFull ? d : 0xFFFFull;
          };
          s.stamps[ea] = f16(ts0, ts1) | (f16(ts1, ts2) << 16) | (f16(ts2, tp) << 32) | (1ull << 52);
          // per part (items it < 4096; the highest index written is
          // B*16 + 20480 + 4095, so a stamps buffer needs B*16 + 24576
          // entries, as tools/dist_stamps.py allocates): stage, strips,
          // publish, strips run, S, merged
          if (it < 4096u) {  // absolute: workgroup start, item start, part end (merged: below)
            s.stamps[(size_t)s.B * 16u + 12288u + it] = ts0;
            s.stamps[(size_t)s.B * 16u + 16384u + it] = tp;
            s.stamps[(size_t)s.B * 16u + 20480u + it] = tk;
          }
          if (it < 4096u)
            s.stamps[(size_t)s.B * 16u + 8192u + it] =
                f16(ts0, tsa) | (f16(tsa, tsb) << 16) | (f16(tsb, ts1) << 32) | (1ull << 59);
          if (it < 4096u)
            s.stamps[(size_t)s.B * 16u + it] = f16(ts0, ts1) | (f16(ts1, ts2) << 16) | (f16(ts2, tp) << 32) |
                                               ((uint64_t)min(__popcll(ran), 63) << 48) | ((uint64_t)S << 54) |
                                               ((uint64_t)merged << 58) | (1ull << 59);
        }
      }
#endif
      if (!merged) {
        __syncthreads();  // the LDS is reused by the next item
        continue;
      }
    }
    // no covered cell: the restatement's convention (-1 everywhere); only the
    // discarded reset-time PRE term can see it
    dist_reload(s, io);
    const int M = fast ? (int)(s_fkey >> 16) : (cov ? (int)(s_key >> 48) : -1);
    const float Mf = (float)M;
    if (fast) {
      cache_serve<kDtThreads>(s, T, ea, s_fkey, ccnt, cM0, s_cdv, s_d, pre_out, dist_obs, count);
    } else {
      if (tid == 0) {  // M unknown (-1) while nothing is covered: every step recomputes it
        const int wu = (int)((s_key >> 16) & 0xFFFF), wv = (int)(s_key & 0xFFFF);
        reinterpret_cast<int2*>(s.dist_mw)[ea] = make_int2(M, pack_witness(wu - pad, wv - pad));
      }
      if (s.dist_ch) {
        // the cache pass: every cell with d >= M - kDistT (strips whose max
        // reaches it; the others only carry their last covered column)
        int cnt = -1;
        // the main pass's list (mode 3: the parts' lists) holds them all
        // (mode 3 / a fused merger of a map without theta0: the part lists)
        const bool parts = mode == 3 || (mode == 2 && S > 1);
        const bool main_ok = kOnePass && (theta0 > 0 || (kPartList && parts)) && s_ccount <= kDistK;
        if (cov && M >= 0 && main_ok) {
          const int thr = M - kDistT, n = s_ccount;
          for (int k = tid; k < n; k += kDtThreads)
            if ((int)s_cdv[k] >= thr) {
              const int j = atomicAdd(&s_kept, 1);
              s.dist_cc[(size_t)ea * kDistK + j] = s_ccell[k];
              s.dist_cd[(size_t)ea * kDistK + j] = s_cdv[k];
            }
          __syncthreads();
          cnt = s_kept;
          dflags |= 1ull << 49;
        } else if (cov && M >= 0) {
          if (idle) stage_cb();  // an idle part merging: the bitboard for the pass
          dflags |= 1ull << 50;
          __syncthreads();  // every thread has read s_ccount
          if (tid == 0) s_ccount = 0;
          __syncthreads();
          const int thr = M - kDistT;
          carry_in(0);
          for (int st = 0; st < nstrips_all; ++st) {
            if (st >= kMaxTrack || s_smax[st] >= thr) {
              strip(st, thr, -1);
              __syncthreads();
              if (s_ccount > kDistK) break;  // overflowed: no cache for this map, the rest is moot
            } else {
              carry_over(st);
            }
          }
          __syncthreads();
          cnt = s_ccount <= kDistK ? s_ccount : -1;
          for (int k = tid; k < (cnt > 0 ? cnt : 0); k += kDtThreads) {
            s.dist_cc[(size_t)ea * kDistK + k] = s_ccell[k];
            s.dist_cd[(size_t)ea * kDistK + k] = s_cdv[k];
          }
        }
        // the strip maxima for the next transform's pruning (skipped strips
        // keep their bound)
        if (cnt > 0)
          for (int st = tid; st < min(nstrips_all, kMaxTrack); st += kDtThreads)
            s.dist_sm[(size_t)ea * kMaxTrack + st] = (uint32_t)min(s_smax[st], 0xFFFF);
        if (tid == 0) {
          reinterpret_cast<int4*>(s.dist_ch + (size_t)ea * 8)[0] = make_int4(cnt, M, 1 << 28, 1 << 28);
          reinterpret_cast<int2*>(s.dist_ch + (size_t)ea * 8)[2] = make_int2(-(1 << 28), -(1 << 28));
        }
      }
    }
    if (!fast) {
      if (post) {
        float* dst = dist_obs + (size_t)ea * E * E;
        for (int t = 5 + tid; t < T; t += kDtThreads)
          dst[t - 5] = dist_value((float)(cov ? s_d[t] : -1), Mf);
      }
      float* pd = pre_out + (size_t)ea * 8;
      if (tid == 0) pd[0] = Mf;
      if (tid < 5) pd[1 + tid] = (float)(cov ? s_d[tid] : -1);
    }
    DSTAMP(ts3);
#ifdef MC_DIST_STAMPS
    if (tid == 0 && s.stamps && ea < (uint32_t)s.B * 16u && mode != 3) {
      auto f16 = [](uint64_t a, uint64_t b) -> uint64_t {
        const uint64_t d = (b - a) >> 4;
        return d < 0xFFFFull ? d : 0xFFFFull;
      };
      const uint64_t ff = min((tsf - ts0) >> 6, (uint64_t)0x1FFF);  // the fast-path attempt, cycles/64
      s.stamps[ea] = f16(ts0, ts1) | (f16(ts1, ts2) << 16) | (f16(ts2, ts3) << 32) | dflags |
                     (fast ? 1ull << 48 : 0ull) | (ff << 51);
    }
    if (tid == 0 && s.stamps && mode == 2 && merged && it < 4096u) {  // the merged part: publish end -> done
      const uint64_t d = (ts3 - ts0) >> 4;
      s.stamps[(size_t)s.B * 16u + 4096u + it] = (d < 0xFFFFFFull ? d : 0xFFFFFFull) | (1ull << 59);
      s.stamps[(size_t)s.B * 16u + 16384u + it] = ts3;
    }
#else
    (void)ts0; (void)ts1; (void)ts2; (void)ts3; (void)tsf; (void)dflags; (void)tsa; (void)tsb; (void)tk;
#endif
    __syncthreads();  // the LDS is reused by the next item
  }
  // the shards' counts (State::dist_shc) = entries, count[1] = workgroups
  // done: the last workgroup to finish zeroes them for the next step's env kernel (every workgroup has
  // read the entry count before it counts itself done; no memset launch per
  // step) and keeps the entry count in count[2] (MC_FIELD_DIST_LISTED); the
  // cache hits count[3] go to count[4] the same way (MC_FIELD_DIST_CACHED)
  if (list && threadIdx.x == 0) {
    uint32_t* cnt = count;
    if (n_items == 0) {
      if (blockIdx.x == 0) {
        cnt[2] = cnt[4] = 0;
        if (s.dist_tot) s.dist_tot[3] += 1ull;
      }
    } else {
      __threadfence();
      if (atomicAdd(cnt + 1, 1u) == gridDim.x - 1) {
        uint32_t nl = 0;
        for (int k = 0; k < kListShards; ++k) nl += atomicExch(s.dist_shc + k * kShardStride, 0u);
        const uint32_t nh = atomicExch(cnt + 3, 0u);
        atomicExch(cnt + 2, nl);
        atomicExch(cnt + 4, nh);
        atomicExch(cnt + 1, 0u);
        if (s.dist_tot) {  // MC_FIELD_DIST_TOTALS: the cache hits were served
          s.dist_tot[0] += nl;
          s.dist_tot[1] += nh;
          s.dist_tot[2] += nl - nh;
          s.dist_tot[3] += 1ull;
        }
      }
    }
  }
}


// static LDS of dist_kernel_t beyond dist_lds_bytes: the top-cell cache list
// (kDistK cells and d), the strip maxima and the scalars
size_t dist_static_lds_bytes() {
  return (size_t)kDistK * (sizeof(int32_t) + sizeof(uint16_t)) + kMaxTrack * sizeof(int) + 64;
}

// Mode 1 of the listed maps: the cache fast path alone, in small workgroups
// with a small LDS (every listed map of a step resident at once: the
// transform kernel's LDS admits two workgroups per CU); a map it cannot
// serve goes to the full list with its theta0 (the exact max of its cached
// cells' d, a lower bound of the new max(d); 0 without a try).
// Build knobs (A/B, profiles/r4/c5_fast/): threads per workgroup and grid.
// A wave per map (64 threads, 512 tiles, grid 4096) was slower: 52.9 vs
// 28.1 us per step at the C5 steady state, the try's time scaling with the
// threads it has.  Round 5 (profiles/r5/fast/, fast2/): early after a reset
// (~14,600 tries per step, ~7 per workgroup one after another) the tries
// are bound by how many maps are in flight: 128 threads, 1,024 staged
// tiles and a grid of 8,192 took the kernel from 57.5 to 40.5 us per step
// (256 threads / 2,048 tiles / 2,048; 64 threads: 47.4), the steady state
// 15.6 -> 16.7 us with the step unchanged (147.1 us both)
#ifndef MC_FAST_THREADS
#define MC_FAST_THREADS 128
#endif
#ifndef MC_FAST_GRID
#define MC_FAST_GRID 8192
#endif
constexpr int kFastThreads = MC_FAST_THREADS;
constexpr int kFastBuf = 128;  // full-list entries a workgroup buffers before one atomic

__global__ __launch_bounds__(kFastThreads) void dist_fast_kernel(DistArgs args) {
  // (DistArgs: post and mode unused; the State and arguments re-read per map,
  // dist_reload)
  State s = args.s;
  DistIO io = args.io;
  const int& pad = io.pad;
  float* const& pre_out = io.pre_out;
  float* const& dist_obs = io.dist_obs;
  const uint32_t* const& list = io.list;
  uint32_t* const& full = io.full;
  extern __shared__ __attribute__((aligned(16))) int s_dyn[];  // the targets' d: [5 + E*E]
  __shared__ uint64_t ft[kFastTiles];
  __shared__ uint16_t cdv[kDistK];
  __shared__ uint32_t s_fkey;
  __shared__ int s_ffail;
  __shared__ uint32_t s_nf, s_fbase, s_nc;
  __shared__ uint2 s_fl[kFastBuf];     // this workgroup's maps for the full list
  __shared__ uint32_t s_cl[kFastBuf];  // this chunk's maps with a cache
  __shared__ uint32_t s_span[6 * kSpan];
  const int tid = threadIdx.x;
  const int T = 5 + s.E * s.E;
  const ListView lv = list_view(s);
  const uint32_t n_items = lv.pre[kListShards];
  uint64_t tk0 = 0;
  DSTAMP(tk0);
  if (tid == 0) s_nf = 0;
  // a contiguous share of the list per workgroup, kFastBuf maps at a time:
  // one thread per map reads its cache header (a map without a cache goes
  // straight to the full list), then the workgroup tries the cache of each
  // map that has one
  auto to_full = [&](uint32_t ea, uint32_t theta) {  // (one thread)
    if (s.dist_rmask) s.dist_rmask[ea] = strip_run_mask(s, pad, ea, (int)theta);
    const uint32_t k = atomicAdd(&s_nf, 1u);
    if (k < (uint32_t)kFastBuf) s_fl[k] = make_uint2(ea, theta);
    else reinterpret_cast<uint2*>(full + 8)[atomicAdd(full, 1u)] = make_uint2(ea, theta);
  };
  const uint32_t per = (n_items + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = min(n_items, blockIdx.x * per), hi = min(n_items, lo + per);
  for (uint32_t c0 = lo; c0 < hi; c0 += kFastBuf) {
    const uint32_t c1 = min(hi, c0 + (uint32_t)kFastBuf);
    if (tid == 0) s_nc = 0;
    __syncthreads();
    for (uint32_t i = c0 + tid; i < c1; i += kFastThreads) {
      const uint32_t ea = list_entry(s, lv, list, i);
      if (s.dist_ch[(size_t)ea * 8] > 0) s_cl[atomicAdd(&s_nc, 1u)] = ea;
      else to_full(ea, 0u);
    }
    __syncthreads();
    const uint32_t nc = s_nc;
    for (uint32_t j = 0; j < nc; ++j) {
      dist_reload(s, io);
      const uint32_t ea = s_cl[j];
      uint64_t tm0 = 0, tm1 = 0, tm2 = 0;
      uint64_t tsv[2] = {0, 0};
      DSTAMP(tm0);
      const int4 h0 = reinterpret_cast<const int4*>(s.dist_ch + (size_t)ea * 8)[0];
      const int2 h1 = reinterpret_cast<const int2*>(s.dist_ch + (size_t)ea * 8)[2];
      const int ccnt = h0.x, cM0 = h0.y;
      const int2 pp = reinterpret_cast<const int2*>(s.pos)[ea];
      for (int t = tid; t < T; t += kFastThreads) s_dyn[t] = -1;
      if (tid == 0) {
        s_fkey = 0;
        s_ffail = 0;
      }
      __syncthreads();
      bool tried = false;
      cache_try<kFastThreads>(s, pad, T, pp.x, pp.y, s.freem + (size_t)ea * s.MT, ccnt, h0.z, h0.w, h1.x, h1.y, ft,
                              s.dist_cc + (size_t)ea * kDistK, s.dist_cd + (size_t)ea * kDistK, cdv, s_dyn, &s_fkey,
                              &s_ffail, tried, s_span,
#ifdef MC_DIST_STAMPS
                              tsv
#else
                              nullptr
#endif
      );
      DSTAMP(tm1);
      dist_reload(s, io);
      const bool served = tried && s_ffail == 0 && (int)(s_fkey >> 16) >= cM0 - kDistT;
      if (served) {
        cache_serve<kFastThreads>(s, T, ea, s_fkey, ccnt, cM0, cdv, s_dyn, pre_out, dist_obs, nullptr);
      } else if (tid == 0) {
        to_full(ea, tried ? (s_fkey >> 16) : 0u);
      }
      DSTAMP(tm2);
#ifdef MC_DIST_STAMPS
      // a served map: the wait from the kernel's start, the try, the serve
      // (the transform kernels stamp the maps they run)
      if (served && tid == 0 && s.stamps && ea < (uint32_t)s.B * 16u) {
        auto f16 = [](uint64_t a, uint64_t b) -> uint64_t {
          const uint64_t d = (b - a) >> 4;
          return d < 0xFFFFull ? d : 0xFFFFull;
        };
        // (diagnostic: the try's phases -- staging, spans + cells, targets)
        s.stamps[ea] = f16(tm0, tsv[0]) | (f16(tsv[0], tsv[1]) << 16) | (f16(tsv[1], tm1) << 32) | (1ull << 48) |
                       (1ull << 51);
        (void)tk0; (void)tm2;
      }
#else
      (void)tm0; (void)tm1; (void)tm2; (void)tk0; (void)tsv;
#endif
      __syncthreads();  // the LDS is reused by the next map
    }
  }
  if (tid == 0 && s_nf > (uint32_t)kFastBuf) s_nf = kFastBuf;  // the rest went to the list directly
  // one atomic per workgroup for the full list (the served count follows
  // from the list lengths, mode 2)
  if (tid == 0) s_fbase = s_nf ? atomicAdd(full, s_nf) : 0u;
  __syncthreads();
  for (uint32_t k = tid; k < s_nf; k += kFastThreads) reinterpret_cast<uint2*>(full + 8)[s_fbase + k] = s_fl[k];
}

// the instantiation whose register chunk holds ceil(RX / kChunks) rows
static hipError_t launch_big(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                             const uint32_t* list, uint32_t* count, unsigned grid, hipStream_t stream);

static hipError_t launch_full(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                              const uint32_t* list, uint32_t* count, unsigned grid, int mode, uint32_t* full,
                              hipStream_t stream) {
  const int RX = s.Wp + 2 * pad, cl = chunk_rows(RX);
  if (RX > kMaxRows) return launch_big(s, pad, post, pre_out, dist_obs, list, count, grid, stream);
  const size_t lds = dt_lds(RX, s.Lp + 2 * pad, s.MT, 5 + s.E * s.E).total;
#define MC_DT(CL)                                                                              \
  do {                                                                                         \
    if (lds > 65536) {                                                                         \
      hipError_t e_ = hipFuncSetAttribute(reinterpret_cast<const void*>(&dist_kernel_t<CL>),   \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
      if (e_ != hipSuccess) return e_;                                                         \
    }                                                                                          \
    hipLaunchKernelGGL(dist_kernel_t<CL>, dim3(grid), dim3(kDtThreads), lds, stream,            \
                       DistArgs{s, DistIO{pad, post, pre_out, dist_obs, list, count, mode, full}}); \
  } while (0)
  if constexpr (kCh == 64) {
    if (cl == 4) MC_DT(4);
    else if (cl == 9) MC_DT(9);
    else MC_DT(13);  // kMaxRows / kCh
  } else {
    if (cl == 8) MC_DT(8);
    else if (cl == 17) MC_DT(17);
    else MC_DT(26);  // kMaxRows / kCh
  }
#undef MC_DT
  return hipGetLastError();
}

// --------------------------------------------------------------------------
// Big maps: extended grids past kMaxRows rows (the reference's own
// Grids/bg2_1073x1073, 1,079 extended rows at egoradius 2).  The transform
// above keeps the map's row bitboard in LDS (RX x RW words: 147 KB at 1079 x
// 1079) next to its strip; a big map's bitboard does not fit beside the
// strip, so this kernel keeps only two 64-column word columns of the map in
// LDS at a time and, per row and word column, the first covered column at or
// right of it (`nxt`, built right to left first: the row pass's nearest
// covered cell right of a strip).  Same strips, same row and column passes
// (a wave of 64 row chunks per column pair), same outputs as mode 0 of
// dist_kernel_t without the top-cell cache (mc_create leaves the cache off
// for these maps).  One workgroup of 1,024 threads per listed map (or per map
// with list == nullptr), one per CU (LDS).
// --------------------------------------------------------------------------
constexpr int kBigThreads = 1024;
constexpr int kBigCh = 64;                    // row chunks per column pair: one wave
constexpr int kBigCL = 17;                    // rows per chunk
constexpr int kBigSP = 34;                    // strip row stride (u16; 17 dwords: distinct banks)
constexpr int kBigMaxRows = kBigCh * kBigCL;  // 1,088 extended rows

struct BigLds {
  size_t nxt, wc, strip, tgt, total;
};
__host__ __device__ inline BigLds big_lds(int Wp, int TC, int T) {
  BigLds L;
  const int RWm = (TC + 7) >> 3;  // u64 words per map row
  L.nxt = (((size_t)(RWm + 1) * Wp * 2) + 15) & ~(size_t)15;
  L.wc = (size_t)2 * Wp * 8;
  L.strip = (size_t)kBigCh * kBigCL * kBigSP * 2;
  L.tgt = ((size_t)T * 4 + 15) & ~(size_t)15;
  L.total = L.nxt + L.wc + L.strip + L.tgt;
  return L;
}

// word column q of the map (u64 per map row: columns 64 q .. 64 q + 63) into
// wc[X], X < Wp: a thread per tile row loads its 8 tiles (two 16-byte pairs of
// block rows) and transposes their bytes into the 8 row words (v_perm, as the
// staging above).  q outside the map: zero words.
__device__ __forceinline__ void big_stage_word(const State& s, const uint64_t* free_t, int q, uint64_t* wc) {
  const int RWm = (s.TC + 7) >> 3;
  for (int ti = opaque_tid(); ti < s.TR; ti += kBigThreads) {
    uint32_t lo[8], hi[8];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const int tj = 8 * q + j;
      uint4 t = make_uint4(0u, 0u, 0u, 0u);
      if (q >= 0 && q < RWm && tj < s.TC) t = *reinterpret_cast<const uint4*>(free_t + tile_index(s.TCS, ti, tj));
      if (tj + 1 >= s.TC) t.z = t.w = 0u;
      lo[j] = t.x;
      hi[j] = t.y;
      lo[j + 1] = t.z;
      hi[j + 1] = t.w;
    }
    const int nr = min(8, s.Wp - 8 * ti);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (r >= nr) break;
      const uint32_t* src = r < 4 ? lo : hi;
      const uint32_t b = (uint32_t)(r & 3);
      const uint32_t sel2 = b | ((4u + b) << 8) | 0x0C0C0000u;
      const uint32_t p01 = __builtin_amdgcn_perm(src[1], src[0], sel2);
      const uint32_t p23 = __builtin_amdgcn_perm(src[3], src[2], sel2);
      const uint32_t p45 = __builtin_amdgcn_perm(src[5], src[4], sel2);
      const uint32_t p67 = __builtin_amdgcn_perm(src[7], src[6], sel2);
      const uint32_t wlo = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
      const uint32_t whi = __builtin_amdgcn_perm(p67, p45, 0x05040100u);
      wc[8 * ti + r] = (uint64_t)wlo | ((uint64_t)whi << 32);
    }
  }
}

__global__ __launch_bounds__(kBigThreads, 1) void dist_big_kernel(State s, int pad, int post, float* __restrict__ pre_out,
                                                                 float* __restrict__ dist_obs,
                                                                 const uint32_t* __restrict__ list,
                                                                 uint32_t* __restrict__ count) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ unsigned long long s_key;
  __shared__ int s_cov;
  const int RX = s.Wp + 2 * pad, RY = s.Lp + 2 * pad;
  const int RWm = (s.TC + 7) >> 3;
  const int E = s.E;
  const int T = post ? 5 + E * E : 5;
  const BigLds LL = big_lds(s.Wp, s.TC, 5 + E * E);
  uint16_t* nxt = reinterpret_cast<uint16_t*>(smem);  // [RWm + 1][Wp]: first covered column >= 64 q (0xFFFF: none)
  uint64_t* wc = reinterpret_cast<uint64_t*>(smem + LL.nxt);  // two word columns [2][Wp]
  uint16_t* G = reinterpret_cast<uint16_t*>(smem + LL.nxt + LL.wc);  // [kBigCh * kBigCL][kBigSP]
  int* s_d = reinterpret_cast<int*>(smem + LL.nxt + LL.wc + LL.strip);
  const int nst = (RY + kStrip - 1) / kStrip;
  ListView lv;
  lv.pre[kListShards] = 0;
  if (list) lv = list_view(s);
  const uint32_t n_items = list ? lv.pre[kListShards] : (uint32_t)gridDim.x;
  for (uint32_t it = blockIdx.x; it < n_items; it += (list ? gridDim.x : n_items)) {
    const int tid = opaque_tid();
    const uint32_t ea = list ? list_entry(s, lv, list, it) : it;
    const uint64_t* free_t = s.freem + (size_t)ea * s.MT;
    const int2 pp = reinterpret_cast<const int2*>(s.pos)[ea];
    const int px = pp.x, py = pp.y;
    auto target = [&](int t, int& u, int& v) {  // as dist_kernel_t (extended coordinates)
      if (t >= 5) {
        const int r = (t - 5) / E, c = (t - 5) - r * E;
        u = px + pad - s.ego + r;
        v = py + pad - s.ego + c;
      } else {
        u = px + (t == 1 ? 1 : (t == 3 ? -1 : 0));
        v = py + (t == 2 ? 1 : (t == 4 ? -1 : 0));
      }
    };
    for (int t = tid; t < T; t += kBigThreads) s_d[t] = -1;
    if (tid == 0) {
      s_key = 0;
      s_cov = 0;
    }
    for (int X = tid; X < s.Wp; X += kBigThreads) nxt[RWm * s.Wp + X] = 0xFFFF;
    // ---- nxt, right to left over the word columns
    int any = 0;
    for (int q = RWm - 1; q >= 0; --q) {
      __syncthreads();  // the last round's wc reads are done
      big_stage_word(s, free_t, q, wc);
      __syncthreads();
      for (int X = tid; X < s.Wp; X += kBigThreads) {
        const uint64_t w = wc[X];
        any |= w != 0;
        nxt[q * s.Wp + X] = w ? (uint16_t)(64 * q + __ffsll((unsigned long long)w) - 1) : nxt[(q + 1) * s.Wp + X];
      }
    }
    if (any) s_cov = 1;
    __syncthreads();
    const bool cov = s_cov != 0;
    // ---- the strips, left to right: wc holds word columns q0, q0 + 1 (slot q & 1)
    int lastL[2] = {-kInf, -kInf};  // last covered extended column left of the strip, rows tid, tid + 1024
    const int chunk = tid & (kBigCh - 1), pair = tid / kBigCh;
    const int u0c = chunk * kBigCL;
    const int nin = max(min(RX - u0c, kBigCL), 0);
    const uint32_t rowmask = nin >= 32 ? ~0u : ((1u << nin) - 1u);
    uint32_t bestkey = 0;
    int bestv = -1;
    const int tu_lo = min(px - 1, px + pad - s.ego), tu_hi = max(px + 1, px + pad + s.ego);
    const int tv_lo = min(py - 1, py + pad - s.ego), tv_hi = max(py + 1, py + pad + s.ego);
    int qs = -2;  // word columns in wc: qs, qs + 1
    for (int st = 0; st < (cov ? nst : 0); ++st) {
      const int c0 = st * kStrip, m0 = c0 - pad;  // extended / map column of the strip's first cell
      const int q0 = m0 >= 0 ? m0 >> 6 : -1;
      if (q0 != qs) {  // advance by one word column (or load both at the start)
        __syncthreads();  // every read of the slot being replaced is done
        if (q0 == qs + 1) {
          big_stage_word(s, free_t, q0 + 1, wc + (size_t)((q0 + 1) & 1) * s.Wp);
        } else {
          big_stage_word(s, free_t, q0, wc + (size_t)(q0 & 1) * s.Wp);
          big_stage_word(s, free_t, q0 + 1, wc + (size_t)((q0 + 1) & 1) * s.Wp);
        }
        qs = q0;
        __syncthreads();
      }
      const int off = m0 - 64 * q0;  // 0..63
      // ---- row pass: g of the strip's 32 cells of each row, 16 u16 pairs
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int u = tid + h * kBigThreads;
        if (u >= kBigCh * kBigCL) continue;
        uint2* grow = reinterpret_cast<uint2*>(G + u * kBigSP);
        const int X = u - pad;
        if (u >= RX || X < 0 || X >= s.Wp) {  // padding rows / the pad ring: no covered cell
#pragma unroll
          for (int k = 0; k < 8; ++k) grow[k] = make_uint2(~0u, ~0u);
          continue;
        }
        const uint64_t wlo = q0 >= 0 ? wc[(size_t)(q0 & 1) * s.Wp + X] : 0ull;
        const uint64_t whi = wc[(size_t)((q0 + 1) & 1) * s.Wp + X];
        const uint32_t sb = (uint32_t)(off ? ((wlo >> off) | (whi << (64 - off))) : wlo);
        // first covered extended column right of the strip (map column m0 + 32 on)
        int firstR = kInf;
        {
          const int p = m0 + 32, qp = p >> 6;  // p >= 0 (pad < 32)
          const uint64_t w = (qp == q0 ? wlo : whi) >> (p & 63);
          if (w) {
            firstR = p + __ffsll((unsigned long long)w) - 1 + pad;
          } else {
            const int nx = qp + 1 <= RWm ? nxt[(qp + 1) * s.Wp + X] : 0xFFFF;
            if (nx != 0xFFFF) firstR = nx + pad;
          }
        }
        const int lc = lastL[h];
        if (sb == 0u) {
          const uint32_t A = (uint32_t)min(c0 - lc, 0xFFFF - kStrip);
          const uint32_t Bd = (uint32_t)min(firstR - c0, 0xFFFF);
          const u16x2 Ap = {(uint16_t)A, (uint16_t)A}, Bp = {(uint16_t)Bd, (uint16_t)Bd};
#pragma unroll
          for (int k = 0; k < kStrip / 4; ++k) {
            const u16x2 c0j = {(uint16_t)(4 * k), (uint16_t)(4 * k + 1)};
            const u16x2 c1j = {(uint16_t)(4 * k + 2), (uint16_t)(4 * k + 3)};
            const u16x2 g0 = __builtin_elementwise_min(Ap + c0j, Bp - c0j);
            const u16x2 g1 = __builtin_elementwise_min(Ap + c1j, Bp - c1j);
            grow[k] = make_uint2(__builtin_bit_cast(uint32_t, g0), __builtin_bit_cast(uint32_t, g1));
          }
        } else if (sb == ~0u) {
#pragma unroll
          for (int k = 0; k < kStrip / 4; ++k) grow[k] = make_uint2(0u, 0u);
          lastL[h] = c0 + 31;
        } else {
#pragma unroll
          for (int j4 = 0; j4 < kStrip; j4 += 4) {
            uint32_t pq[2];
#pragma unroll
            for (int h2 = 0; h2 < 2; ++h2) {
              const int j = j4 + 2 * h2;
              int gg[2];
#pragma unroll
              for (int k = 0; k < 2; ++k) {
                const uint32_t le = sb & (0xFFFFFFFFu >> (31 - (j + k)));
                const uint32_t ge = sb & (0xFFFFFFFFu << (j + k));
                const int left = le ? c0 + 31 - __clz(le) : lc;
                const int right = ge ? c0 + __ffs(ge) - 1 : firstR;
                gg[k] = min(min(c0 + j + k - left, right - (c0 + j + k)), 0xFFFF);
              }
              pq[h2] = (uint32_t)gg[0] | ((uint32_t)gg[1] << 16);
            }
            grow[j4 >> 2] = make_uint2(pq[0], pq[1]);
          }
          lastL[h] = c0 + 31 - __clz(sb);
        }
      }
      __syncthreads();
      // ---- column pass (as dist_kernel_t's, 64 chunks of a column pair per wave)
      int u0 = u0c;
      asm volatile("" : "+v"(u0));
      const uint32_t* g32 = reinterpret_cast<const uint32_t*>(G) + u0 * (kBigSP / 2) + pair;
      u16x2 tp[kBigCL], sd[kBigCL];
      u16x2 pm = kNone2, sm = kNone2;
#pragma unroll
      for (int i = 0; i < kBigCL; ++i) {
        const u16x2 g = __builtin_bit_cast(u16x2, g32[i * (kBigSP / 2)]);
        const u16x2 uu = splat2(u0 + i);
        tp[i] = __builtin_elementwise_sub_sat(__builtin_elementwise_add_sat(g, kRowOff2), uu);
        sd[i] = __builtin_elementwise_add_sat(g, uu);
        pm = __builtin_elementwise_min(pm, tp[i]);
        sm = __builtin_elementwise_min(sm, sd[i]);
      }
      __syncthreads();  // every G read of the strip is done: the next row pass may write
      u16x2 run = excl_prefix_min64(pm), sfx = excl_suffix_min64(sm);
#pragma unroll
      for (int i = kBigCL - 1; i >= 0; --i) {
        sfx = __builtin_elementwise_min(sfx, sd[i]);
        sd[i] = __builtin_elementwise_sub_sat(sfx, splat2(u0 + i));
      }
      uint32_t klo = 0, khi = 0;
#pragma unroll
      for (int i = 0; i < kBigCL; ++i) {
        const u16x2 uu = splat2(u0 + i);
        run = __builtin_elementwise_min(run, tp[i]);
        const u16x2 up = __builtin_elementwise_sub_sat(__builtin_elementwise_add_sat(run, uu), kRowOff2);
        const uint32_t d = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(up, sd[i])) &
                           (uint32_t)__builtin_amdgcn_sbfe((int)rowmask, i, 1);
        tp[i] = __builtin_bit_cast(u16x2, d);
        klo = max(klo, (d << 16) | (uint32_t)(u0 + i));
        khi = max(khi, (d & 0xFFFF0000u) | (uint32_t)(u0 + i));
      }
      const int v = c0 + 2 * pair;
      if (v < RY && klo > bestkey) {
        bestkey = klo;
        bestv = v;
      }
      if (v + 1 < RY && khi > bestkey) {
        bestkey = khi;
        bestv = v + 1;
      }
      const bool keep = v + 1 >= tv_lo && v <= tv_hi && u0 + kBigCL > tu_lo && u0 <= tu_hi;
      if (keep) {
        for (int t = 0; t < T; ++t) {
          int tu, tv;
          target(t, tu, tv);
          if ((tv == v || tv == v + 1) && tu >= u0 && tu < u0 + kBigCL && tu < RX) {
            uint32_t val = 0;
#pragma unroll
            for (int i = 0; i < kBigCL; ++i) val = (u0 + i == tu) ? __builtin_bit_cast(uint32_t, tp[i]) : val;
            s_d[t] = (int)(tv == v ? (val & 0xFFFFu) : (val >> 16));
          }
        }
      }
    }
    const int vmax = bestv >= 0 ? (int)(bestkey >> 16) : -1;
    if (cov && vmax >= 0) {
      const int ubest = (int)(bestkey & 0xFFFF), vbest = bestv;
      const int far = abs(ubest - (px + pad)) + abs(vbest - (py + pad));
      atomicMax(&s_key, ((unsigned long long)vmax << 48) | ((unsigned long long)far << 32) |
                            ((unsigned long long)ubest << 16) | (unsigned long long)vbest);
    }
    __syncthreads();
    const int M = cov ? (int)(s_key >> 48) : -1;
    const float Mf = (float)M;
    if (tid == 0) {
      const int wu = (int)((s_key >> 16) & 0xFFFF), wv = (int)(s_key & 0xFFFF);
      reinterpret_cast<int2*>(s.dist_mw)[ea] = make_int2(M, pack_witness(wu - pad, wv - pad));
    }
    if (post) {
      float* dst = dist_obs + (size_t)ea * E * E;
      for (int t = 5 + tid; t < T; t += kBigThreads) dst[t - 5] = dist_value((float)(cov ? s_d[t] : -1), Mf);
    }
    float* pd = pre_out + (size_t)ea * 8;
    if (tid == 0) pd[0] = Mf;
    if (tid < 5) pd[1 + tid] = (float)(cov ? s_d[tid] : -1);
    __syncthreads();  // the LDS is reused by the next item
  }
  // the work list's bookkeeping, as dist_kernel_t's (mode 0 with a list)
  if (list && threadIdx.x == 0) {
    uint32_t* cnt = count;
    if (n_items == 0) {
      if (blockIdx.x == 0) {
        cnt[2] = cnt[4] = 0;
        if (s.dist_tot) s.dist_tot[3] += 1ull;
      }
    } else {
      __threadfence();
      if (atomicAdd(cnt + 1, 1u) == gridDim.x - 1) {
        uint32_t nl = 0;
        for (int k = 0; k < kListShards; ++k) nl += atomicExch(s.dist_shc + k * kShardStride, 0u);
        const uint32_t nh = atomicExch(cnt + 3, 0u);
        atomicExch(cnt + 2, nl);
        atomicExch(cnt + 4, nh);
        atomicExch(cnt + 1, 0u);
        if (s.dist_tot) {
          s.dist_tot[0] += nl;
          s.dist_tot[1] += nh;
          s.dist_tot[2] += nl - nh;
          s.dist_tot[3] += 1ull;
        }
      }
    }
  }
}

static hipError_t launch_big(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                             const uint32_t* list, uint32_t* count, unsigned grid, hipStream_t stream) {
  const size_t lds = big_lds(s.Wp, s.TC, 5 + s.E * s.E).total;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&dist_big_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  // a list: one resident workgroup per CU strides over it (LDS: one per CU)
  const unsigned g = list ? (grid < 256u ? grid : 256u) : grid;
  hipLaunchKernelGGL(dist_big_kernel, dim3(g), dim3(kBigThreads), lds, stream, s, pad, post, pre_out, dist_obs, list,
                     count);
  return hipGetLastError();
}

size_t dist_lds_bytes(const State& s, int pad) {
  if (s.Wp + 2 * pad > kMaxRows) return big_lds(s.Wp, s.TC, 5 + s.E * s.E).total;
  return dt_lds(s.Wp + 2 * pad, s.Lp + 2 * pad, s.MT, 5 + s.E * s.E).total;
}

// extended rows the distance transform takes (dist_big_kernel past
// kMaxRows) / that the LDS-bitboard transform, its split parts and the
// top-cell cache take
int dist_max_rows() { return kBigMaxRows; }
int dist_cache_max_rows() { return kMaxRows; }

hipError_t launch_dist(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                       hipStream_t stream) {
  return launch_full(s, pad, post, pre_out, dist_obs, nullptr, nullptr, (unsigned)((size_t)s.B * s.N), 0,
                     nullptr, stream);
}

// --------------------------------------------------------------------------
// POST terms without a full transform.  Sensing only adds covered cells, so
// d only decreases and max(d) only decreases; the env kernel keeps M
// (S.dist_mw) unless a new cell came closer than M to the witness, a cell
// with d == M (then d(witness) is still M, and no cell exceeds M).  The
// targets (the E x E crop and the 5 end cells of the next step) are near the
// robot, so the env kernel settles their d from the agent's staged block
// (mc_env_kernel.hip dist_window) and lists only the maps with an unknown M
// or a target the block cannot settle.  With the top-cell cache, the listed
// maps first try the cache (mode 1) and the rest run split over workgroups
// (mode 2; `full`: the full list), finalised by mode 3 when split over more
// than one part; without it, each listed map runs whole (mode 0).  The grids
// are fixed (hipGraph capture) and stride.
// --------------------------------------------------------------------------
hipError_t launch_dist_listed(const State& s, int pad, float* pre_out, float* dist_obs,
                              uint32_t* list, uint32_t* count, uint32_t* full, hipStream_t stream) {
  const size_t maps = (size_t)s.B * s.N;
  const unsigned grid = (unsigned)(maps < 2048 ? maps : 2048);
  if (!full || !s.dist_ch)
    return launch_full(s, pad, 1, pre_out, dist_obs, list, count, grid, 0, nullptr, stream);
  const unsigned fgrid = (unsigned)(maps < MC_FAST_GRID ? maps : MC_FAST_GRID);
  hipLaunchKernelGGL(dist_fast_kernel, dim3(fgrid), dim3(kFastThreads), (size_t)(5 + s.E * s.E) * 4, stream,
                     DistArgs{s, DistIO{pad, 1, pre_out, dist_obs, list, count, 1, full}});
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // grids of about the resident workgroups (two per CU); mode 2 has at most
  // kSplitSlots items when it splits (a 2048-workgroup grid measured the
  // same: 202.3 vs 202.3 us per C5 steady step, profiles/r4/c5_grid/)
  const unsigned g2 = (unsigned)(maps < (size_t)kSplitSlots ? maps : (size_t)kSplitSlots);
  e = launch_full(s, pad, 1, pre_out, dist_obs, nullptr, count, g2, 2, full, stream);
  if (e != hipSuccess || kFused) return e;
  return launch_full(s, pad, 1, pre_out, dist_obs, nullptr, count, g2 < 256 ? g2 : 256, 3, full, stream);
}

}  // namespace mc
