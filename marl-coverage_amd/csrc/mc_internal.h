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
  int16_t axis;   // bit 0 -- 0: major axis is x (rows), 1: y (columns); bit 1: march
                  // from the per-start table (no common pattern for this beam)
  int16_t sign;   // +1 / -1 along the major axis
  int32_t msign;  // +1 / -1 / 0: direction of a minor-axis move
  uint32_t bits;  // the step bits shared by every start (unless axis bit 1)
};
static_assert(sizeof(Beam) == 16, "Beam is 16 bytes");


// Bit maps are stored as 8x8-cell tiles: one u64 per tile, bit 8*r + c =
// cell (8*ti + r, 8*tj + c).  Tiles are grouped 4 x 4 into 128-byte blocks
// (one cache line; row-major blocks, row-major tiles inside a block:
// tile_index), so an agent's window block of TW x TW tiles touches few lines
// (at C2 about 3 per plane instead of 5 with plain tile rows).  Cells of an
// edge tile beyond the padded grid are obstacles in grid_neg and never set in
// the other maps; the padding tiles of the last blocks likewise.
//
// Everything a kernel needs, passed by value.  Layout (all device memory):
//   grid_neg/grid_pos  u64 [G][MT]      tiles of grid < 0 / grid > 0
//   freem/obstm        u64 [B][N][MT]   per-agent _free_pad/_obst_pad
//   vis                u64 [B][MT]      _visited (union of free maps)
// (each mask array has one more tile at its end that is always zero)
// with MT = TRS * TCS * 16 tiles per map in tile_index order.
//   pos                i32 [B][N][2]       (_xinds, _yinds)
struct State {
  int B, N, Wp, Lp, G;
  int TR, TC;              // tile rows / columns of a map: ceil(Wp/8), ceil(Lp/8)
  int TRS, TCS;            // 4x4-tile block rows / columns: ceil(TR/4), ceil(TC/4)
  int MT;                  // tiles per map (TRS * TCS * 16)
  int H;                   // sensing half-width (>= egoradius)
  int TW;                  // window tiles per side (window_tiles(H))
  uint32_t mg_TW2, mg_TW, mg_LcE, mg_E, mg_nb;  // magic reciprocals: n / d == umulhi(n, mg_d)
  int ego, E, Lc;          // egoradius, obs side, obs layers
  int pad;                 // max(egoradius, mini_map_rad): the extended grid's ring (dec_grid_rl.py:78)
  int sensor, nbeams, sq_r;
  double pen, term, dincr;
  int maxsteps, comm_r, sst, auto_reset, grid_mode;
  int dist;                // dist_reward: add the pre-sense distance terms
  uint64_t seed;
  uint32_t env0, grid0;     // global ids of env 0 / pool grid 0 (mc_config env_offset / grid_offset)

  const uint64_t* grid_neg;
  const uint64_t* grid_pos;
  const int32_t* numfree;
  const Beam* beams;
  const uint64_t* beam_bits;  // [nbeams][bcmax] minor-move bits per start coordinate
  int bcmax;                  // max(Wp, Lp)
  int beam_kmax;              // max Beam::K (<= H): march steps of a pass
  int beam_kmin;              // min Beam::K: steps k <= beam_kmin are in range for every beam
  // 1: every beam marches the same minor steps (Beam::bits) from every start
  // coordinate a robot can occupy, up to the step where it reaches the
  // grid's border (an obstacle, so the march ends there): the march needs no
  // beam_bits load (mc_set_beam_table checks this on the host)
  int beam_common;
  // beam_common: the cells every beam visits at step 1 (always reached: step 0
  // is the robot's own free cell), and the robot cell, as a 3x3 mask around
  // the robot (bit 3*(dx+1) + (dy+1)); the march marks them once per agent
  // instead of once per ray (0 = no premark, the march marks step 1)
  uint32_t beam_k1;
  // Fan march of a dense beam set (mc_env_kernel.hip fan_march; built by
  // mc_set_beam_table, off when fan_nsec + fan_nspec == 0).  fan_data: the
  // spread / expand LUTs (kFanLutBytes), fan_nsec / 2 sector-pair records of
  // 2 (fan_kt + 1) words (the two sectors of one line, interleaved: words 0, 1
  // their FAN_* class bits, words 2k, 2k + 1 their step-k entries) and
  // fan_nspec special-beam records of 8 words (FAN_SPECIAL);
  // fan_words words in all (a multiple of 4), copied into LDS each launch.
  int fan_nsec, fan_nspec, fan_kt, fan_words;
  const uint32_t* fan_data;
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
  const float* dist_pre;   // dist_reward: [B][N][8] max(d), d of the 5 end cells (mc_dist.hip)
  // dist_reward: [B][N] (M, witness) of each free map: M = max(d) over the
  // extended grid (-1: unknown), witness = a cell with d == M (map
  // coordinates, (x << 16) | (y & 0xFFFF), signed halves).  The env kernel
  // sets M = -1 when sensing covers a cell closer than M to the witness (or
  // the env resets); otherwise M is unchanged (mc_dist.hip).
  int32_t* dist_mw;
  // dist_reward POST outputs of the env kernel's window search (mc_env_kernel
  // dist_window): the caller's float32 obs layer [B][N][E][E] and the header
  // of the full transform's work list (count at [0], entries from [5]:
  // mc_dist.hip dist_kernel_t)
  float* dist_obs_out;
  uint32_t* dist_cnt;
  // the work list's append counters, one per shard (env e appends to shard
  // e % kListShards; counters kShardStride words apart), and the entries per
  // shard: shard k's entries start at dist_cnt[5 + k * dist_cap]
  uint32_t* dist_shc;
  uint32_t dist_cap;
  // dist_reward: cumulative POST counters since mc_create (MC_FIELD_DIST_TOTALS):
  // maps listed, served by the top-cell cache, fully transformed, POST launches
  unsigned long long* dist_tot;
  // the split transform's full list (mc_dist.hip modes 1 / 2; null without
  // it): the env kernel empties it for the step (its count read by the last
  // step's mode 2 is done by then)
  uint32_t* dist_full;
  // dist_reward top-cell cache (mc_dist.hip; null when off, e.g. with map
  // sharing): per map kDistK cells (witness packing) and their d, and a
  // header [8]: count (-1: none), M0 (max(d) when the cells were taken),
  // the box (x0, y0, x1, y1, map coordinates) that holds every cell covered
  // since the cells' d were last made exact (x1 < x0: empty).  The cells are
  // every cell with d >= M0 - kDistT then; the env kernel grows the box by
  // each step's sensing windows and drops the cache on a reset.
  int32_t* dist_cc;
  int32_t* dist_cd;
  int32_t* dist_ch;
  // with the cache: per map, an upper bound of max(d) over each 32-column
  // strip of the extended grid ([B][N][kDistStrips] u32: the strip maxima of
  // the last full transform; d only decreases), valid while the cache is
  // (32-bit words: a split transform's parts hand them over by `sc1` dword
  // stores, mc_dist.hip)
  uint32_t* dist_sm;
  // with the cache: the split full transform's per-map partials (mc_dist.hip
  // modes 2 / 3; zero between uses): the best key [B][N]; by full-list index
  // (< kDistGSlots) and part (< kDistGParts) the candidate count each part
  // published and its candidates [kDistGSlots][kDistGParts][kDistK] (cell, d)
  unsigned long long* dist_gkey;
  uint32_t* dist_gcnt;
  // by full-list index: 1 + the largest own maximum of the parts whose
  // candidate list overflowed (0: none), for maps split without a cache
  // bound (theta0 = 0; mc_dist.hip part lists)
  uint32_t* dist_govf;
  int2* dist_gcand;
  uint32_t* dist_pcnt;  // [B][N] parts of a split map done this launch (mode 2 fused; zero between uses)
  // [B][N] the strips a listed map's split transform runs (bit st: not
  // pruned; mc_dist.hip strip_run_mask), written when the map goes to the full
  // list, read by every part of the next launch to balance the parts
  unsigned long long* dist_rmask;
  // episode record, written when an env reports done (before an auto-reset
  // clears the counters): percent_covered() and _currstep at the end
  double* ep_pc;
  int32_t* ep_len;
};

constexpr int kMaxItemsPerLane = 2;  // staged (agent, tile) items per lane
#ifndef MC_DIST_K  // build-time A/B knobs (tools/build_variants.py)
#define MC_DIST_K 512
#endif
#ifndef MC_DIST_T
#define MC_DIST_T 20
#endif
constexpr int kDistK = MC_DIST_K;    // top-cell cache: cells per map
constexpr int kDistGSlots = 256;      // full-list entries a split transform can split (mc_dist.hip kSplitSlots / 2)
constexpr int kDistGParts = 8;        // candidate segments per entry: one per part (mc_dist.hip kMaxParts)
constexpr int kListShards = 8;        // dist work-list append counters (one address took every env's atomic)
constexpr int kShardStride = 32;      // u32 words between them (a 128-B line each)
constexpr int kDistStrips = 64;      // strips whose maxima the cache keeps (extended grids up to 2048 columns)
constexpr int kDistT = MC_DIST_T;    // ... with d >= M0 - kDistT

// word index of tile (ti, tj) in a map (0 <= ti < 4*TRS, 0 <= tj < 4*TCS)
__host__ __device__ inline uint32_t tile_index(int TCS, int ti, int tj) {
  return ((uint32_t)((ti >> 2) * TCS + (tj >> 2)) << 4) | (uint32_t)((ti & 3) << 2) |
         (uint32_t)(tj & 3);
}

// Lidar marks are made in "row form" (one u32/u64 per window row: the march's
// address and bit are then one add and one shift), so a window row must fit
// 64 bits: TW <= 8, i.e. H <= 27.  An agent's rows are 8*TW + 1 apart (odd:
// the same row of different agents falls on different LDS banks).
constexpr int kMaxWindowTiles = 8;

// Window tiles per side for half-width H.  The staged "extended window" of an
// agent is the cells [x0-H-1, x0+H+1] around its pre-move cell (the +1 margin
// covers every post-move window); its tile block starts at tile
// floor((x0-H-1)/8), so 8*TW >= 7 + (2H+3).
__host__ __device__ constexpr int window_tiles(int H) { return (2 * H + 3 + 7 + 7) / 8; }

// floor(n / d) == umulhi(n, magic(d)) for 2 <= d < 2^16 and n * d < 2^32;
// d == 1 (2^32 does not fit) is encoded as 0 and handled by the caller
__host__ __device__ constexpr uint32_t magic_div(uint32_t d) {
  return d <= 1 ? 0u : (uint32_t)((0x100000000ull + d - 1) / d);
}

// Words of one row plane of the env kernel (mc_env_kernel.hip row_word):
// 32-bit rows are agent-interleaved with an odd stride N | 1 (row lx of agent
// a is word lx * (N | 1) + a), 64-bit rows agent-major, 8*TW + 1 apart.
__host__ __device__ inline int row_plane_words(int N, int TW, int rowbytes) {
  return rowbytes == 4 ? 8 * TW * (N | 1) : N * (8 * TW + 1);
}

// Fan march (mc_env_kernel.hip fan_march): sectors of up to kFanS adjacent
// beams of one octant class march together.  Entry of step k (u32):
// bits 0-5 lo + 32 (signed minor offset of the sector's first cell), bits 6-10
// D (bit j: beam j+1 sits one cell past beam j), bits 16-21 the beams still in
// range (K >= k).  LUTs: spread[D][A] (cells lit by the live beams A) and
// expand[D][F] (beams on the cells F), 2048 bytes each.
constexpr int kFanS = 6;
constexpr int kFanLutBytes = 4096;
// Sector record word 0: FAN_COLS (major axis y: a column line), FAN_NEG
// (major sign -1), FAN_SPECIAL (the sector holds a beam with start-dependent
// bits: its slot in bits 3-5, its special record in bits 8+).  Special
// record (8 words): beam, class bits, minor sign, K, first and last minor
// start whose bits differ from the common ones.
enum : uint32_t { FAN_COLS = 1u, FAN_NEG = 2u, FAN_SPECIAL = 4u };

// LDS bytes of the fan region (replaces the beam records): the fan data and
// the per-(agent, special beam) pair records.  The fan's column planes share
// the tile region (env_lds_bytes; mc_env_kernel.hip carve).
__host__ __device__ inline size_t fan_lds_bytes(int N, int nspec, int kt, int words) {
  return (size_t)words * 4 + (size_t)N * nspec * 2 * (kt + 1) * 4;
}

// LDS bytes of one env slot of the env kernel (host + device use the same carve).
// rowbytes: 4 when a window row (8*TW cells) fits a u32, else 8.  fanb: the
// fan region's bytes (0: beam records instead).
__host__ __device__ inline size_t env_lds_bytes(int N, int TW, int nbeams, int rowbytes, size_t fanb = 0) {
  // fold, oold, fp tiles; the square sensor (nbeams == 0) also neg, pos, op;
  // the fan's column planes neg / marks / seen overlay this region
  const size_t rowplanes = (((size_t)3 * row_plane_words(N, TW, rowbytes) * rowbytes) + 15) & ~(size_t)15;
  size_t b = (size_t)(nbeams > 0 ? 3 : 6) * N * TW * TW * 8;
  if (fanb && b < rowplanes) b = rowplanes;
  b += rowplanes;  // neg / marks / seen rows
  b += fanb ? ((fanb + 15) & ~(size_t)15) : (size_t)(nbeams > 0 ? nbeams : 1) * 16;  // fan region / beams
  b += (((size_t)N * 8 * 4) + 15) & ~(size_t)15;       // x0, y0, x, y, bx, by, dist M / witness
  b += 64;                                             // scalars
  b += ((size_t)N + 15) & ~(size_t)15;                 // actions
  b += 64 * (size_t)rowbytes;                          // per-lane sink words (lidar marks)
  return b;
}

// the env slot of a State (lidar beams or fan region)
__host__ __device__ inline size_t state_lds_bytes(const State& s, int rowbytes) {
  const bool fan = s.sensor == 0 && s.fan_nsec + s.fan_nspec > 0;
  return env_lds_bytes(s.N, s.TW, s.sensor == 0 ? s.nbeams : 0, rowbytes,
                       fan ? fan_lds_bytes(s.N, s.fan_nspec, s.fan_kt, s.fan_words) : 0);
}

// Byte stride between the env slots of a workgroup: skewed by 20 LDS banks so
// the two slots' row planes do not fall on the same banks.
__host__ __device__ inline size_t slot_stride(size_t slot_lds) {
  return ((slot_lds + 255) & ~(size_t)255) + 80;
}

// Compile-time shape of an env kernel instantiation: fields > 0 are baked in
// (loop bounds, divisions and LDS offsets fold to constants and the march
// unrolls); 0 leaves the field to the runtime State.  The launcher picks a
// specialised instantiation only when the runtime State matches it exactly.
// LC: obs layers of an EGO shape (3; 4 with dijkstra_input, whose layer 3 the
// dijkstra kernel writes after the env kernel, or with dist_reward, whose
// layer 3 is the float buffer: 0 in the uint8 obs).  DS: an EGO shape's
// dist_reward flag (baked in).  FN / FS / FW: a dense-beam shape's fan
// march -- sector slots, special beams and fan words (mc_set_beam_table's
// build_fan; its trip count is KM): the fan's LDS offsets (carve) then fold
// to constants instead of living in SGPRs across the kernel.  BW: a bench
// instantiation -- square padded grids of side BW (the tile geometry and the
// beam-bit row length fold to constants) with the bench's episode flags (no
// comm graph, grids kept on reset, auto-reset on).
template <int N_, int H_, int NB_, int EGO_, int KM_, int KN_ = 0, int LC_ = 3, int DS_ = 0, int FN_ = 0,
          int FS_ = 0, int FW_ = 0, int BW_ = 0>
struct Shape {
  static constexpr int N = N_, H = H_, NB = NB_, EGO = EGO_, KM = KM_, KN = KN_, LC = LC_, DS = DS_;
  static constexpr int FN = FN_, FS = FS_, FW = FW_, BW = BW_;
  __host__ __device__ static bool matches(const State& s) {
    return (N_ == 0 || s.N == N_) && (H_ == 0 || s.H == H_) &&
           (NB_ == 0 || (s.sensor == 0 && s.nbeams == NB_)) &&
           (EGO_ == 0 || (s.ego == EGO_ && s.Lc == LC_ && (s.dist != 0) == (DS_ != 0))) &&
           (KM_ == 0 || (s.sensor == 0 && s.beam_kmax == KM_)) &&
           (KN_ == 0 || (s.sensor == 0 && s.beam_kmin == KN_)) &&
           (FN_ == 0 || (s.fan_nsec == FN_ && s.fan_nspec == FS_ && s.fan_words == FW_ && s.fan_kt == KM_)) &&
           (BW_ == 0 || (s.Wp == BW_ && s.Lp == BW_ && s.comm_r == 0 && s.grid_mode == 0 && s.auto_reset == 1));
  }
};

// overwrite the baked-in fields of a kernel's State copy with constants
template <class SH>
__device__ __forceinline__ void specialize(State& s) {
  if constexpr (SH::N > 0) s.N = SH::N;
  if constexpr (SH::H > 0) {
    s.H = SH::H;
    s.TW = window_tiles(SH::H);
    s.mg_TW = magic_div(window_tiles(SH::H));
    s.mg_TW2 = magic_div(window_tiles(SH::H) * window_tiles(SH::H));
  }
  if constexpr (SH::NB > 0) {
    s.sensor = 0;
    s.nbeams = SH::NB;
    s.mg_nb = magic_div(SH::NB);
  }
  if constexpr (SH::NB > 0 && SH::NB < 64) {  // sparse beams: never the fan march (build_fan)
    s.fan_nsec = 0;
    s.fan_nspec = 0;
  }
  if constexpr (SH::EGO > 0) {
    s.ego = SH::EGO;
    s.E = 2 * SH::EGO + 1;
    s.Lc = SH::LC;
    s.mg_E = magic_div(2 * SH::EGO + 1);
    s.mg_LcE = magic_div(SH::LC * (2 * SH::EGO + 1));
  }
  if constexpr (SH::KM > 0) s.beam_kmax = SH::KM;
  if constexpr (SH::BW > 0) {  // (mc_capi.hip mc_create / mc_set_beam_table derive the same)
    constexpr int T8 = (SH::BW + 7) / 8, T32 = (T8 + 3) / 4;
    s.Wp = s.Lp = SH::BW;
    s.TR = s.TC = T8;
    s.TRS = s.TCS = T32;
    s.MT = T32 * T32 * 16;
    s.bcmax = SH::BW;
    s.comm_r = 0;
    s.grid_mode = 0;
    s.auto_reset = 1;
  }
  if constexpr (SH::FN > 0) {
    s.fan_nsec = SH::FN;
    s.fan_nspec = SH::FS;
    s.fan_words = SH::FW;
    s.fan_kt = SH::KM;
  }
  if constexpr (SH::KN > 0) s.beam_kmin = SH::KN;
  if constexpr (SH::EGO > 0) s.dist = SH::DS;  // an EGO shape bakes in its dist_reward flag
  // (LC 3 / 4 leaves no room for minimap layers: mini_map_rad = 0, pad = ego)
  if constexpr (SH::EGO > 0 && SH::LC <= 4) s.pad = SH::EGO;
}

}  // namespace mc
