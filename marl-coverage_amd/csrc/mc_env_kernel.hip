// mc_env_kernel.hip — the step / reset kernel of the batched coverage env.
//
// Hot path restated from ExistentialRobotics/MARL-Coverage
//   Environments/dec_grid_rl.py  DecGridRL.step :91-169, reset :449-531
//   Environments/Sensors/lidar.py LidarSensor.getMeasurement :16-65
//   Environments/Sensors/squaresensor.py SquareSensor.getMeasurement :15-37
//
// Maps live in HBM as 8x8-cell u64 tiles (mc_internal.h).  A workgroup runs
// EPW envs ("slots"), LPE = NT / EPW lanes each; small envs (the BASELINE
// configs) pack two envs into one wave.  Per env and step:
//   round trip 1  positions, actions, per-env scalars
//   round trip 2  for every agent the TW x TW tile block around its pre-move
//                 cell (the extended window [x0-H-1, x0+H+1] rounded out to
//                 tiles): grid neg/pos tiles, its free/obst tiles, the union
//                 (visited) tiles — TW coalesced runs of TW words per plane.
//                 The +1 margin covers every post-move window, so the moves,
//                 the beam march and the merge need no further loads.
//   LDS compute   moves (slot-serial in robot order); lidar sensing as a beam
//                 march over "row form" planes (one WT word per window row,
//                 scattered from the tiles at stage time) with ds_or marks,
//                 gathered back into tiles afterwards; square sensing directly
//                 on tiles; merge with popcounts — agents' blocks share the
//                 global tile grid, so the union dedup is a tile-for-tile AND
//   stores        changed tiles (plain stores: one writer per agent tile),
//                 newly covered union bits (global_atomic_or: agents' blocks
//                 overlap), positions, counters, reward, done, obs
// All float64 arithmetic is the reference's: rewards are assembled in
// reference order; the beam's float64 `+=` chain is encoded bit-exactly in
// the host-built step bits (mc_internal.h, struct Beam).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>
#include <type_traits>

#include "mc_device.h"

namespace mc {

#include "mc_diag.h"  // STAMP(k): phase stamps of -DMC_STAMPS diagnostic builds

// n / d via the magic reciprocal of mc_internal.h (magic == 0 encodes d == 1)
__device__ __forceinline__ int udiv(int n, uint32_t magic) {
  return magic ? (int)__umulhi((uint32_t)n, magic) : n;
}

__device__ __forceinline__ int rdlane(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

struct Scal {
  double pen;          // move penalties, accumulated in robot order
  uint64_t dist_fail;  // dist_reward: agents with a target the window search left unsettled
  uint64_t moved;      // robots present in the reference's _robot_pad
  uint32_t cnt_free;   // newly set bits over all agents' free maps
  uint32_t cnt_vis;    // newly covered union cells (the obs reward)
  int32_t grid;
  uint32_t ep;
  int32_t do_reset;
  int32_t path;        // the step's branch flags (kPath*), read back after it
  uint64_t dist_hit;   // dist_reward: agents whose witness cell got closer than M
  uint64_t zero;       // always 0: the merge's dedup reads it for agents whose block misses the tile
};
static_assert(sizeof(Scal) <= 64, "Scal must fit its 64-byte LDS slot");

// Scal::path bits
constexpr int kPathActive = 1, kPathResetReq = 2, kPathSentReset = 4, kPathSentinel = 8;

// the lidar marches by sectors (fan_march) rather than by rays
__device__ __forceinline__ bool fan_on(const State& s) { return s.sensor == 0 && s.fan_nsec + s.fan_nspec > 0; }

// One env slot's LDS.  Tile planes are [N][TW][TW] u64 in the agent's block
// coordinates.  Row planes are [N][8*TW+1] WT: row lx of agent a's block, bit ly
// = cell (8*bx + lx, 8*by + ly); the lidar march and the moves read them.
// negr: grid < 0; fldr: the cells the agent has seen (dense beam sets: cells
// a ray need not mark again); fpr: every cell a ray visited this step -- its
// free marks are the cells with grid >= 0, its obstacle marks the others
// (a ray marks free cells up to the first obstacle, and that obstacle), so
// one plane and one target per mark, split by the grid tile in the merge.
template <typename WT>
struct Lds {
  uint64_t *neg, *pos, *fold, *oold, *fp, *op;
  WT *negr, *fldr, *fpr;
  // fan march (dense beams): column planes (word ly of agent a at
  // row_word(a, ly), bit lx = cell (8*bx + lx, 8*by + ly)) of neg, marks and
  // seen cells, the same distances apart as negr / fpr / fldr; fan data
  // (LUTs, sector records, special-beam records) and the per-(agent,
  // special beam) entries.  Null without the fan.
  WT *cneg, *cmark, *cseen;
  uint32_t *fan, *fspec;
  Beam* beams;
  int32_t *x0, *y0, *x, *y;  // pre-move / post-move cells
  int32_t *bx, *by;          // tile-block origin (tile units) of each agent
  int32_t *dm, *dw;          // dist_reward: M and witness of each agent's free map
  Scal* sc;
  uint8_t* act;
  WT* sink;                  // [64] target of lidar marks a lane does not make
};

template <typename WT>
__device__ __forceinline__ Lds<WT> carve(char* smem, const State& s) {
  Lds<WT> L;
  const int tiles = s.N * s.TW * s.TW;
  const int rows = row_plane_words(s.N, s.TW, (int)sizeof(WT));
  uint64_t* p = reinterpret_cast<uint64_t*>(smem);
  // the grid tile planes (neg, pos) and the obstacle-mark plane (op) serve
  // the square sensor only: a lidar slot carves fold, oold, fp (env_lds_bytes)
  const bool square = s.sensor != 0;
  const bool fan = fan_on(s);
  const size_t rowplanes = (((size_t)3 * rows * sizeof(WT)) + 15) & ~(size_t)15;
  // fan: the column planes overlay the tile planes -- cneg / cseen are dead
  // after the march, cmark (read by gather_marks, which writes fp) lies past
  // fp (rows * sizeof(WT) >= tiles * 8: TW <= 8) and under fold / oold,
  // which the merge writes after gather_marks
  L.fp = fan ? p : p + 2 * tiles;
  L.fold = fan ? p + tiles : p;
  L.oold = fan ? p + 2 * tiles : p + tiles;
  L.neg = square ? p + 3 * tiles : nullptr;
  L.pos = square ? p + 4 * tiles : nullptr;
  L.op = square ? p + 5 * tiles : nullptr;
  L.cneg = L.cmark = L.cseen = nullptr;
  if (fan) {
    L.cneg = reinterpret_cast<WT*>(smem);
    L.cmark = L.cneg + rows;
    L.cseen = L.cmark + rows;
  }
  size_t tb = (size_t)(square ? 6 : 3) * tiles * 8;
  if (fan && tb < rowplanes) tb = rowplanes;
  char* q = smem + tb;
  L.negr = reinterpret_cast<WT*>(q);
  L.fpr = L.negr + rows;
  L.fldr = L.fpr + rows;
  q += rowplanes;
  L.fan = L.fspec = nullptr;
  L.beams = reinterpret_cast<Beam*>(q);
  if (fan) {
    L.fan = reinterpret_cast<uint32_t*>(q);
    L.fspec = L.fan + s.fan_words;
    q += (fan_lds_bytes(s.N, s.fan_nspec, s.fan_kt, s.fan_words) + 15) & ~(size_t)15;
  } else {
    q += (size_t)(s.nbeams > 0 ? s.nbeams : 1) * 16;
  }
  L.x0 = reinterpret_cast<int32_t*>(q);
  L.y0 = L.x0 + s.N;
  L.x = L.y0 + s.N;
  L.y = L.x + s.N;
  L.bx = L.y + s.N;
  L.by = L.bx + s.N;
  L.dm = L.by + s.N;
  L.dw = L.dm + s.N;
  q += (((size_t)s.N * 8 * 4) + 15) & ~(size_t)15;
  L.sc = reinterpret_cast<Scal*>(q);
  q += 64;
  L.act = reinterpret_cast<uint8_t*>(q);
  q += ((size_t)s.N + 15) & ~(size_t)15;
  L.sink = reinterpret_cast<WT*>(q);
  return L;
}

// Row planes of 32-bit rows (TW <= 4: every BASELINE config but C4) are
// agent-interleaved: window row lx of agent a is word lx * N + a.  The rays
// of one march instruction sit in about N * 8 rows of the slot's agents;
// interleaved, agent a's rows own the banks = a (mod N) and its consecutive
// rows are N banks apart, while with agent-major rows, a * (8 TW + 1) + lx,
// two agents' rows collide whenever a + lx == a' + lx' (mod 32).  A
// bank-conflict simulation of the C2 march: 2.5x -> 1.5x the conflict-free
// read cycles; measured C2 9.35 -> 9.25 us.  64-bit rows keep the
// agent-major order (8-byte words interleaved by 8 agents would fall on 4
// banks per agent: C4 283 -> 305 us).
template <typename WT>
__device__ __forceinline__ int row_step(const State& s) { return sizeof(WT) == 4 ? (s.N | 1) : 1; }
template <typename WT>
__device__ __forceinline__ int row_word(const State& s, int a, int lx) {
  return sizeof(WT) == 4 ? lx * (s.N | 1) + a : a * (8 * s.TW + 1) + lx;
}

// one env slot of the workgroup
template <int NT, int EPW, typename WT>
struct Ctx {
  static constexpr int LPE = NT / EPW;            // lanes per env
  static constexpr int KI = kMaxItemsPerLane;     // staged tiles per lane
  static constexpr int RPL = EPW == 1 ? 2 : 3;  // beams per lane per pass (C4 A/B: 3, 4 or 6 are slower)
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

// staged (agent, tile) items of this lane; old HBM tiles stay in registers
// from stage to store
template <int KI>
struct Items {
  int a[KI];
  int gi[KI], gj[KI];   // global tile coordinates
  bool in[KI];          // tile inside the map (and item live)
  uint64_t f[KI], o[KI], u[KI];     // old free / obst / union tiles (raw loads)
  uint64_t nf[KI], no[KI], nu[KI];  // newly set bits
  uint64_t mf[KI], mo[KI];          // lidar: this step's free / obstacle marks (gather_marks)
  uint64_t n[KI];                   // grid < 0 tiles (raw load; outside the map: all ones after stage_scatter)
  uint64_t p[KI];                   // grid > 0 tiles (square sensor)
  int ti[KI], tj[KI];               // tile within the agent's block
  bool masks;                       // f / o / u were loaded (else known zero)
};

template <typename WT>
__device__ __forceinline__ void lds_or(WT* p, WT v) {
  if constexpr (sizeof(WT) == 4) atomicOr((unsigned int*)p, (unsigned int)v);
  else atomicOr((unsigned long long*)p, (unsigned long long)v);
}

// Dense beam sets (C4: 360 beams, 1 degree apart) mark every cell near the
// robot, and the nearest obstacles, from dozens of rays at once, and those
// same-address LDS ORs serialise; nearly all of those cells are in the
// agent's maps already (the grid is static: a cell once seen free or
// obstacle is marked the same way again).  So with >= 64 beams the march
// also reads the agent's seen cells (old free | obstacle, row plane fldr)
// and skips their marks: the merge keeps only new bits, and a seen free
// cell is in the union, so no union delta needs it.  Sparse sets (C2) gain
// less than the extra reads cost (measured: 10.9 vs 10.0 us at C2).
__device__ __forceinline__ bool dense_beams(const State& s) { return s.sensor == 0 && s.nbeams >= 64; }

// tile_index (mc_internal.h) for non-negative tile coordinates below 2^24:
// one full-rate v_mul_u32_u24 instead of a quarter-rate v_mul_lo_u32
__device__ __forceinline__ uint32_t tile_index24(int TCS, int ti, int tj) {
  return ((__umul24((uint32_t)(ti >> 2), (uint32_t)TCS) + (uint32_t)(tj >> 2)) << 4) |
         (uint32_t)((ti & 3) << 2) | (uint32_t)(tj & 3);
}

// element i of a per-env / per-agent array.  O32: every such array's byte
// offsets fit 32 bits (launch-checked with the maps), so the address is the
// uniform base plus a 32-bit offset (global_* saddr form, no 64-bit address
// arithmetic per access)
template <bool O32, typename T>
__device__ __forceinline__ T& el(T* base, uint32_t i) {
  if constexpr (O32) {
    using B = std::conditional_t<std::is_const_v<T>, const char, char>;  // keep const, stay a global pointer
    return *reinterpret_cast<T*>(reinterpret_cast<B*>(base) + (size_t)(i * (uint32_t)sizeof(T)));
  } else {
    return base[i];
  }
}

// tile idx of a map array.  O32: the launcher checked that every byte offset
// of the arrays fits 32 bits, so the address is the array base (uniform,
// SGPRs) plus a 32-bit offset (one VGPR: global_load's saddr form, no
// 64-bit address arithmetic per load)
template <bool O32>
__device__ __forceinline__ uint64_t ld_tile(const uint64_t* base, uint32_t idx) {
  if constexpr (O32) return *reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(base) + (size_t)(idx << 3));
  else return base[idx];
}

// --------------------------------------------------------------------------
// stage: one round trip for every staged tile (masks known zero after reset)
// --------------------------------------------------------------------------
// Compiled shapes with at most 8 robots and one wave per workgroup: the
// robots' pre-move cells and actions are broadcast to every lane of the slot
// by v_readlane right after round trip 1 (no LDS round trip, no barrier), so
// the tile-block origins of round trip 2 and the moves come from registers.
template <int NS>
struct Front {
  uint32_t xy[NS > 0 ? NS : 1];  // pre-move cell, x | y << 16
  int act[NS > 0 ? NS : 1];
  int bx[NS > 0 ? NS : 1], by[NS > 0 ? NS : 1];  // tile-block origins
};

// R[a] for a runtime index a < NS, as a select chain (the empty asm keeps
// the compiler from folding the chain back into an indexed scratch array)
template <int NS>
__device__ __forceinline__ int pick(const int (&R)[NS], int a) {
  int v = R[0];
#pragma unroll
  for (int i = 1; i < NS; ++i) {
    v = a == i ? R[i] : v;
    asm volatile("" : "+v"(v));
  }
  return v;
}

// the value v of lane lane0 + i of this lane's slot, read with wave-uniform
// lane indices (v_readlane) and selected by slot
template <int NT, int EPW, typename WT>
__device__ __forceinline__ int slot_lane(const Ctx<NT, EPW, WT>& C, int v, int i) {
  static_assert(NT == 64 || EPW == 1, "one wave per workgroup, or the first wave of one env");
  if constexpr (EPW == 1) return rdlane(v, i);
  else {
    static_assert(EPW == 2, "two slots per wave");
    const int lo = rdlane(v, i), hi = rdlane(v, 32 + i);
    return C.lane0 ? hi : lo;
  }
}

// QUAD (NS divides 4): round trip 1 loaded robot sub % NS into every lane,
// so lanes 4q + i of every quad hold robot i and one DPP quad_perm broadcast
// (full rate, no LDS) gives every lane robot i's value
template <int NS>
struct FrontQuad {
  static constexpr bool ok = NS > 0 && 4 % NS == 0;
};

template <int NS>
__device__ __forceinline__ int quad_bcast(int v, int i) {  // i: a constant once unrolled
  switch (i) {  // quad_perm [i, i, i, i]
    case 0: return __builtin_amdgcn_mov_dpp(v, 0x00, 0xF, 0xF, false);
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x55, 0xF, 0xF, false);
    case 2: return __builtin_amdgcn_mov_dpp(v, 0xAA, 0xF, 0xF, false);
    default: return __builtin_amdgcn_mov_dpp(v, 0xFF, 0xF, 0xF, false);
  }
}

template <int NT, int EPW, typename WT, int NS>
__device__ __forceinline__ void front_regs(const State& s, const Ctx<NT, EPW, WT>& C, int x, int y, int act,
                                           Front<NS>& F) {
  const int xy = (int)((uint32_t)x | ((uint32_t)y << 16));
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    if constexpr (FrontQuad<NS>::ok) {
      F.xy[i] = (uint32_t)quad_bcast<NS>(xy, i);
      F.act[i] = quad_bcast<NS>(act, i);
    } else {
      F.xy[i] = (uint32_t)slot_lane(C, xy, i);
      F.act[i] = slot_lane(C, act, i);
    }
    F.bx[i] = ((int)(F.xy[i] & 0xFFFFu) - s.H - 1) >> 3;  // arithmetic shift: floor
    F.by[i] = ((int)(F.xy[i] >> 16) - s.H - 1) >> 3;
  }
}

// round trip 2, issue: addresses, then every load of the lane back to back
// with no exec-mask branches (tiles outside the map read tile 0 and are
// replaced in stage_scatter).  NS > 0: block origins from F (registers),
// else from LDS (L.bx / L.by, written after round trip 1).
template <int NT, int EPW, typename WT, int KI, bool O32 = false, int NS = 0>
__device__ __forceinline__ void stage_load(const State& s, const Ctx<NT, EPW, WT>& C, int g,
                                           bool load_masks, Items<KI>& I, const Front<NS>* F = nullptr) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int TW = s.TW, TW2 = TW * TW;
  const int items = s.N * TW2;
  const uint32_t mt = (uint32_t)s.MT;
  const uint32_t gb = __umul24((uint32_t)g, mt);  // this env's grid in the pool (tiles)
  const bool square = s.sensor == 1;
  // 32-bit word indices (mc_create bounds every map array below 2^32 words);
  // products of 24-bit factors are single v_mul_u32_u24
  uint32_t gt[KI], fw[KI], vk[KI];
  int bxa[KI], bya[KI];
  const uint32_t eN = (uint32_t)C.e * (uint32_t)s.N;
  const uint32_t vw = __umul24((uint32_t)C.e, mt);
  const uint32_t zf = (uint32_t)s.B * (uint32_t)s.N * mt, zv = (uint32_t)s.B * mt;  // the zero tiles
  // every item's block origin read first (one LDS round trip for all items)
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    const bool it = idx < items;
    const int a = it ? udiv(idx, s.mg_TW2) : 0;
    const int rem = idx - a * TW2;
    I.ti[k] = udiv(rem, s.mg_TW);
    I.tj[k] = rem - I.ti[k] * TW;
    I.a[k] = a;
    if constexpr (NS > 0) {
      bxa[k] = pick<NS>(F->bx, a);
      bya[k] = pick<NS>(F->by, a);
    } else {
      bxa[k] = L.bx[a];
      bya[k] = L.by[a];
    }
  }
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    const int gi = bxa[k] + I.ti[k], gj = bya[k] + I.tj[k];
    I.gi[k] = gi;
    I.gj[k] = gj;
    I.in[k] = (idx < items) & ((unsigned)gi < (unsigned)s.TR) & ((unsigned)gj < (unsigned)s.TC);
    gt[k] = tile_index24(s.TCS, I.in[k] ? gi : 0, I.in[k] ? gj : 0);
    // tiles outside the map read the mask arrays' zero tile (mc_create)
    fw[k] = I.in[k] ? __umul24(eN + (uint32_t)I.a[k], mt) + gt[k] : zf;
    vk[k] = I.in[k] ? vw + gt[k] : zv;
  }
  // grid tiles first: the moves and the march need only them, so the mask
  // tiles (needed from the merge on) stay in flight meanwhile (loads return
  // in order; the compiler waits only for what each use needs)
#pragma unroll
  for (int k = 0; k < KI; ++k) I.n[k] = ld_tile<O32>(s.grid_neg, gb + gt[k]);
  if (square) {
#pragma unroll
    for (int k = 0; k < KI; ++k) I.p[k] = ld_tile<O32>(s.grid_pos, gb + gt[k]);
  }
  if (load_masks) {
#pragma unroll
    for (int k = 0; k < KI; ++k) {
      I.f[k] = ld_tile<O32>(s.freem, fw[k]);
      I.o[k] = ld_tile<O32>(s.obstm, fw[k]);
      I.u[k] = ld_tile<O32>(s.vis, vk[k]);
    }
  } else {
#pragma unroll
    for (int k = 0; k < KI; ++k) I.f[k] = I.o[k] = I.u[k] = 0;
  }
  I.masks = load_masks;
}

// 8x8 bit-matrix transpose of a tile (bit 8r + c <-> bit 8c + r)
__device__ __forceinline__ uint64_t transpose8(uint64_t x) {
  uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
  x ^= t ^ (t << 7);
  t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
  x ^= t ^ (t << 14);
  t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
  return x ^ t ^ (t << 28);
}

// round trip 2, landing: the grid tiles into the row planes (and the tile
// planes for the square sensor; the column planes for the fan march)
template <int NT, int EPW, typename WT, int KI>
__device__ __forceinline__ void stage_scatter(const State& s, const Ctx<NT, EPW, WT>& C, Items<KI>& I) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int items = s.N * s.TW * s.TW;
  const bool square = s.sensor == 1;
#ifdef MC_STAMPS
  STAMP(11);  // loads issued
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(12);  // loads landed
#endif
  uint8_t* nb = reinterpret_cast<uint8_t*>(L.negr);
  uint8_t* fb = reinterpret_cast<uint8_t*>(L.fldr);
  const bool known = dense_beams(s);
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const bool in = I.in[k];
    const int idx = C.sub + k * LPE;
    if (idx < items) {
      const uint64_t nt = in ? I.n[k] : ~0ull;  // outside the map: blocked (isInBounds)
      I.n[k] = nt;
      if (square) {
        L.neg[idx] = nt;
        L.pos[idx] = in ? I.p[k] : 0ull;
      }
      // scatter the tile's 8 row bytes into the row plane (byte tj of rows
      // 8*ti .. 8*ti+7 of the agent's block)
      const size_t off = (size_t)row_word<WT>(s, I.a[k], 8 * I.ti[k]) * sizeof(WT) + I.tj[k];
      const size_t rs = (size_t)row_step<WT>(s) * sizeof(WT);  // one window row
      const uint64_t ft = (known && I.masks && in) ? (I.f[k] | I.o[k]) : 0ull;
#pragma unroll
      for (int r = 0; r < 8; ++r) nb[off + r * rs] = (uint8_t)(nt >> (8 * r));
      if (known) {  // the cells the agent has seen (old free | obstacle tiles), the same way
#pragma unroll
        for (int r = 0; r < 8; ++r) fb[off + r * rs] = (uint8_t)(ft >> (8 * r));
      }
      if (fan_on(s)) {
        // fan march: the column planes too -- byte ti of words 8*tj .. 8*tj+7
        // are the transposed tile's bytes
        uint8_t* cb = reinterpret_cast<uint8_t*>(L.cneg);
        uint8_t* sb = reinterpret_cast<uint8_t*>(L.cseen);
        const size_t coff = (size_t)row_word<WT>(s, I.a[k], 8 * I.tj[k]) * sizeof(WT) + I.ti[k];
        const uint64_t nT = transpose8(nt), fT = transpose8(ft);
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          cb[coff + r * rs] = (uint8_t)(nT >> (8 * r));
          sb[coff + r * rs] = (uint8_t)(fT >> (8 * r));
        }
      }
    }
  }
}

template <int NT, int EPW, typename WT, int KI, bool O32 = false>
__device__ __forceinline__ void stage(const State& s, const Ctx<NT, EPW, WT>& C, int g,
                                      bool load_masks, Items<KI>& I) {
  stage_load<NT, EPW, WT, KI, O32>(s, C, g, load_masks, I);
  stage_scatter<NT, EPW, WT, KI>(s, C, I);
}

// old mask tiles of item k (zero outside the map, where nothing is stored:
// such items loaded the arrays' zero tile; without mask loads they are 0)
template <int KI>
__device__ __forceinline__ void old_tiles(const Items<KI>& I, int k, uint64_t& f, uint64_t& o,
                                          uint64_t& u) {
  f = I.f[k];
  o = I.o[k];
  u = I.u[k];
}

// the old free / obstacle tiles into LDS (obs of an env that does not step)
template <int NT, int EPW, typename WT, int KI>
__device__ __forceinline__ void stage_fold(const State& s, const Ctx<NT, EPW, WT>& C,
                                           const Items<KI>& I) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const int items = s.N * s.TW * s.TW;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    if (idx < items) {
      uint64_t f, o, u;
      old_tiles<KI>(I, k, f, o, u);
      C.L.fold[idx] = f;
      C.L.oold[idx] = o;
    }
  }
}

// lidar mark rows start empty (LDS stores: issued while loads are in flight)
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void zero_marks(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  if (s.sensor != 0) return;
  const bool fan = fan_on(s);
  for (int r = C.sub; r < row_plane_words(s.N, s.TW, (int)sizeof(WT)); r += LPE) {
    C.L.fpr[r] = 0;
    if (fan) C.L.cmark[r] = 0;
  }
}

// tile (ti, tj) of agent a gathered from a row plane (the inverse scatter):
// byte r of the tile = byte tj of word w0 + r * rs (row 8 ti + r; rs = N)
#ifndef MC_GATHER_BYTES  // build knob (A/B): 0 extracts byte tj of 64-bit rows by shifts
#define MC_GATHER_BYTES 1
#endif
template <typename WT>
__device__ __forceinline__ uint64_t gather_tile(const WT* rows, int w0, int rs, int tj) {
  if constexpr (sizeof(WT) == 4) {
    // v_perm_b32: two rows' byte tj into bytes 0, 1; then two such pairs
    const uint32_t sel = (uint32_t)tj | ((uint32_t)(4 + tj) << 8) | 0x0C0C0000u;
    uint32_t h[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      h[q] = __builtin_amdgcn_perm((uint32_t)rows[w0 + (2 * q + 1) * rs], (uint32_t)rows[w0 + 2 * q * rs], sel);
    const uint32_t lo = __builtin_amdgcn_perm(h[1], h[0], 0x05040100u);
    const uint32_t hi = __builtin_amdgcn_perm(h[3], h[2], 0x05040100u);
    return (uint64_t)lo | ((uint64_t)hi << 32);
  } else if constexpr (MC_GATHER_BYTES != 0) {
    // 64-bit rows: byte tj of the 8 rows by byte loads (the stage's scatter
    // writes them the same way), packed by v_perm -- instead of a 64-bit
    // shift, a mask and a 64-bit shift-or per row
    const uint8_t* rb = reinterpret_cast<const uint8_t*>(rows + w0) + tj;
    const int rsb = rs * (int)sizeof(WT);
    uint32_t b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) b[r] = rb[r * rsb];
    const uint32_t p01 = __builtin_amdgcn_perm(b[1], b[0], 0x0C0C0400u);
    const uint32_t p23 = __builtin_amdgcn_perm(b[3], b[2], 0x0C0C0400u);
    const uint32_t p45 = __builtin_amdgcn_perm(b[5], b[4], 0x0C0C0400u);
    const uint32_t p67 = __builtin_amdgcn_perm(b[7], b[6], 0x0C0C0400u);
    const uint32_t lo = __builtin_amdgcn_perm(p23, p01, 0x05040100u);
    const uint32_t hi = __builtin_amdgcn_perm(p67, p45, 0x05040100u);
    return (uint64_t)lo | ((uint64_t)hi << 32);
  } else {
    uint64_t t = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) t |= (uint64_t)((rows[w0 + r * rs] >> (8 * tj)) & (WT)0xFF) << (8 * r);
    return t;
  }
}

// --------------------------------------------------------------------------
// moves: updateRobotPos in robot order (dec_grid_rl.py:128-145, :171-204).
// Lane lane0+i = robot i of the slot.  Occupancy is the live position set: a
// robot may enter a cell vacated earlier in this step and is blocked by a
// higher-index robot that has not moved yet (:186,190-199,310).  The grid
// test reads the staged window (1 outside the map = isInBounds).
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
    const int lx = x + dx - 8 * L.bx[C.sub], ly = y + dy - 8 * L.by[C.sub];
    gblk = (int)((L.negr[row_word<WT>(s, C.sub, lx)] >> ly) & (WT)1);
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

#ifndef MC_RPL_SHAPE  // A/B knob: 0 keeps 2 rays per lane per pass for every one-env-per-workgroup shape
#define MC_RPL_SHAPE 1
#endif
#ifndef MC_ABL  // diagnostic ablations (timing only, results wrong): 1 no dist_window, 2 no dist rows in
#define MC_ABL 0  // merge, 3 no overlap dedup in merge, 4 no obs, 5 no sensing march
#endif
#ifndef MC_MOVES_SERIAL  // A/B knob: 1 keeps the serial broadcast rounds (moves) at C5
#define MC_MOVES_SERIAL 0
#endif

// Same moves for a compile-time agent count NS > 8 with one env per
// workgroup (C5: 16 robots), by a fixed point instead of N serial broadcast
// rounds.  Robot i moves iff its action is a move (0..3), its target is not
// blocked (grid < 0, out of bounds) and no robot sits on the target at its
// turn: robots j < i at their final cells, robots j > i at their starting
// cells (:186,190-199,310).  So robot i's outcome depends only on the
// outcomes of robots j < i: iterating "moves = ok0 and target not occupied
// under the previous iterate's cells" fixes robot 0 after one round, robot 1
// after two, ..., and the true outcome is the iteration's only fixed point.
// Starting from "every unblocked robot moves", a step without a conflict
// between robots ends after one round and its check.  Lane i = robot i of
// the first wave; each round is NS compares per lane against the robots'
// cells read as scalars (v_readlane), one ballot.
template <int NT, int EPW, typename WT, int NS>
__device__ __forceinline__ void moves_par(const State& s, const Ctx<NT, EPW, WT>& C, double pen_unit) {
  static_assert(EPW == 1 && NS > 0 && NS <= 64, "one env per workgroup, compile-time robots <= 64");
  const Lds<WT>& L = C.L;
  const int i = C.sub;  // lane of the first wave
  const bool live = i < NS;
  const int x = live ? L.x0[i] : 0, y = live ? L.y0[i] : 0;
  const int act = live ? (int)L.act[i] : 255;
  const int dx = (act == 0) - (act == 2), dy = (act == 1) - (act == 3);
  bool blk = true;
  if (live && act < 4) {
    const int lx = x + dx - 8 * L.bx[i], ly = y + dy - 8 * L.by[i];
    blk = ((L.negr[row_word<WT>(s, i, lx)] >> ly) & (WT)1) != 0;
  }
  const bool acts = live && act <= 3;  // not 0..3: no updateRobotPos call, no penalty
  const bool ok0 = acts && !blk;
  // cells packed x | y << 16 (padded-grid coordinates, < 2^16; a target is
  // inside the -1 border, so no coordinate is negative)
  const uint32_t X = (uint32_t)x | ((uint32_t)y << 16);
  const uint32_t T = (uint32_t)(x + dx) | ((uint32_t)(y + dy) << 16);
  uint32_t XA[NS], TA[NS];
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    XA[j] = (uint32_t)rdlane((int)X, j);
    TA[j] = (uint32_t)rdlane((int)T, j);
  }
  uint64_t cm = __ballot(ok0);  // bit j: robot j moves (the iterate)
  bool c = ok0;
  for (int it = 0; it <= NS; ++it) {  // (at most NS + 1 rounds; ~2 in practice)
    bool occ = false;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const uint32_t pj = ((cm >> j) & 1ull) ? TA[j] : XA[j];  // robot j's final cell under the iterate
      occ |= (j < i ? pj : XA[j]) == T;                         // (j == i: X != T for a move)
    }
    c = ok0 && !occ;
    const uint64_t nm = __ballot(c);
    if (nm == cm) break;
    cm = nm;
  }
  if (live) {
    L.x[i] = c ? x + dx : x;
    L.y[i] = c ? y + dy : y;
  }
  // reward += -collision_penalty per failed move, in robot order (:203)
  const int fails = __popcll(__ballot(acts && !c));
  if (i == 0) {
    double pen = 0.0;
    for (int k = 0; k < fails; ++k) pen += pen_unit;
    L.sc->pen = pen;
    L.sc->moved = L.sc->moved | cm;
  }
}

// Same moves for a compile-time agent count NS <= 8: every lane of the slot
// replays the robot-order loop on all robots' data in registers (no
// cross-lane traffic); lane 0 publishes the result.
template <int NT, int EPW, typename WT, int NS>
__device__ __forceinline__ void moves_regs(const State& s, const Ctx<NT, EPW, WT>& C, double pen_unit) {
  const Lds<WT>& L = C.L;
  int X[NS], Y[NS], DX[NS], DY[NS];
  bool acts[NS], blk[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    X[i] = L.x0[i];
    Y[i] = L.y0[i];
    const int act = L.act[i];
    acts[i] = act <= 3;  // not 0..3: no updateRobotPos call, no penalty
    DX[i] = (act == 0) - (act == 2);
    DY[i] = (act == 1) - (act == 3);
    const int lx = X[i] + DX[i] - 8 * L.bx[i], ly = Y[i] + DY[i] - 8 * L.by[i];
    blk[i] = (L.negr[row_word<WT>(s, i, lx)] >> ly) & (WT)1;
  }
  double pen = 0.0;
  uint64_t moved = L.sc->moved;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int tx = X[i] + DX[i], ty = Y[i] + DY[i];
    bool occ = false;
#pragma unroll
    for (int j = 0; j < NS; ++j) occ |= X[j] == tx && Y[j] == ty;
    const bool ok = acts[i] && !blk[i] && !occ;
    if (ok) {
      X[i] = tx;
      Y[i] = ty;
      moved |= 1ull << i;
    }
    if (acts[i] && !ok) pen += pen_unit;  // reward += -collision_penalty (:203)
  }
  if (C.sub == 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      L.x[i] = X[i];
      L.y[i] = Y[i];
    }
    L.sc->pen = pen;
    L.sc->moved = moved;
  }
}

// Moves from registers (Front): robot i's target-cell bit (grid < 0 or out of
// bounds) was loaded by lane lane0 + i next to round trip 2 and is shared by
// a ballot; every lane of the slot replays the robot-order loop; lane 0
// publishes the result.  Same semantics as moves_regs.
template <int NT, int EPW, typename WT, int NS>
__device__ __forceinline__ void moves_front(const State& s, const Ctx<NT, EPW, WT>& C, const Front<NS>& F,
                                            bool tgt_blk, uint32_t txy, int act_own, uint64_t moved,
                                            double pen_unit) {
  const Lds<WT>& L = C.L;
  // QUAD: every lane holds its quad's robot (sub % NS): its packed target
  // and flags (bit 0 blocked, bit 1 acts) go to the loop by quad_perm
  const int fl = (tgt_blk ? 1 : 0) | (act_own <= 3 ? 2 : 0);
  uint64_t bm = 0;
  if constexpr (!FrontQuad<NS>::ok) bm = slot_ballot(C, C.sub < NS && tgt_blk);  // bit i: robot i's target is blocked
  uint32_t XY[NS];
#pragma unroll
  for (int i = 0; i < NS; ++i) XY[i] = F.xy[i];
  double pen = 0.0;
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    bool acts, blk;
    uint32_t t;
    if constexpr (FrontQuad<NS>::ok) {
      const int fi = quad_bcast<NS>(fl, i);
      acts = (fi & 2) != 0;
      blk = (fi & 1) != 0;
      t = (uint32_t)quad_bcast<NS>((int)txy, i);
    } else {
      const int act = F.act[i];
      acts = act <= 3;  // not 0..3: no updateRobotPos call, no penalty
      blk = (bm >> i) & 1ull;
      const int dx = (act == 0) - (act == 2), dy = (act == 1) - (act == 3);
      t = (uint32_t)((int)(XY[i] & 0xFFFFu) + dx) | ((uint32_t)((int)(XY[i] >> 16) + dy) << 16);
    }
    bool occ = false;
#pragma unroll
    for (int j = 0; j < NS; ++j) occ |= XY[j] == t;  // live positions (:186,190-199,310)
    const bool ok = acts && !blk && !occ;
    if (ok) {
      XY[i] = t;
      moved |= 1ull << i;
    }
    if (acts && !ok) pen += pen_unit;  // reward += -collision_penalty (:203)
  }
  if (C.sub == 0) {
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      L.x[i] = (int)(XY[i] & 0xFFFFu);
      L.y[i] = (int)(XY[i] >> 16);
    }
    L.sc->pen = pen;
    L.sc->moved = moved;
  }
}

// --------------------------------------------------------------------------
// lidar march (lidar.py:34-63), integer form.  The major coordinate moves
// exactly +-1 per step; the minor cell moves by msign at the steps flagged in
// the host-built beam_bits word for this (beam, start coordinate), which
// encodes the reference's float64 `+=` chain bit-exactly (mc_internal.h).
// Every cell of a beam lies within Chebyshev K <= H of the post-move robot,
// which is within 1 of the staged window's centre: no window check is needed
// (mc_set_beam_table rejects K > H).  Row planes: the cell's word is one add,
// its bit one shift.
// --------------------------------------------------------------------------
typedef __attribute__((address_space(3))) char lds_char;

// A ray's cell is packed as P = (row word's LDS address << 6) | column: one
// add advances it, P >> 6 addresses the row word, and the shift amount of
// 1 << P is taken mod the word width by the hardware.
struct Ray {
  uint32_t bits;     // minor-move bit per step (K <= 31)
  uint32_t P;        // packed current cell
  uint32_t d0, d1;   // packed major step / minor step (added when the bit is set)
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
  const int row = row_word<WT>(s, a, xa - 8 * L.bx[a]);
  const int col = ya - 8 * L.by[a];
  const int RB = row_step<WT>(s) * (int)sizeof(WT) * 64;  // one window row in P units
  // the row word's LDS address: P >> 6 is the neg-plane word's address
  // itself (no per-step base add)
  const uint32_t plane = (uint32_t)(uintptr_t)(const lds_char*)(const char*)L.negr;
  R.P = ((plane + (uint32_t)row * (uint32_t)sizeof(WT)) << 6) | (uint32_t)col;
  const bool ax = (bm.axis & 1) == 0;
  R.d0 = (uint32_t)(ax ? bm.sign * RB : bm.sign);
  R.d1 = (uint32_t)(ax ? bm.msign : bm.msign * RB);
  R.K = R.live ? bm.K : -1;
  // the beam's own step bits unless its pattern depends on the start
  // coordinate (Beam::axis bit 1: mc_set_beam_table; C4: 2 of 360 beams)
  R.bits = !R.live ? 0u
           : (s.beam_common || !(bm.axis & 2)) ? bm.bits
                                               : (uint32_t)s.beam_bits[(size_t)b * s.bcmax + (ax ? ya : xa)];
  return R;
}

__device__ __forceinline__ void ray_advance(Ray& R, int k) {
  const uint32_t m = 0u - ((R.bits >> k) & 1u);
  R.P += R.d0 + (m & R.d1);
}

// the word of plane `plane` (a row plane of L, the same shape as negr) in
// the ray's current row
template <typename WT>
__device__ __forceinline__ const WT* ray_word(const Lds<WT>& L, const WT* plane, const Ray& R) {
  const lds_char* p = (const lds_char*)(uintptr_t)(R.P >> 6) + (plane - L.negr) * (int)sizeof(WT);
  return reinterpret_cast<const WT*>((const char*)p);
}

// Branch-free mark: every lane issues one ds_or per ray and step; a lane with
// nothing to mark ORs into its own sink word (no bank conflicts, no exec-mask
// branches).  Re-marking an already free cell is harmless (OR).
// `dup`: the lane's previous ray (the adjacent beam) marks the same cell at
// this step, so this one skips its atomic (near the robot adjacent beams share
// cells: fewer same-address LDS atomics).  `premarked`: the cell is one of the
// step-1 cells sense() marked once per agent (State::beam_k1).  Returns
// whether the ray marked.
template <typename WT, int KN>
__device__ __forceinline__ bool ray_mark(const Lds<WT>& L, Ray& R, int k, WT nrow, WT frow,
                                         uint32_t sink_m, bool dup, bool frow_valid, bool premarked) {
  // KN: a compile-time lower bound of every beam's K (steps k <= KN need no
  // range test)
  const bool on = R.live && (k <= KN || k <= R.K);
  const WT bit = (WT)1 << (R.P & (8 * sizeof(WT) - 1));
  const bool hit = (nrow & bit) != 0;  // oc[int(cx), int(cy)] < 0: the beam ends here
  dup |= (frow & bit) != 0;  // a cell the agent has seen: its mark is known (frow: 0 unless dense)
  // mark-plane word = row word + a constant; a lane with nothing to mark
  // selects its sink word less that constant (sink_m), so the constant rides
  // in the instruction's offset field.  (Two exec-masked ORs at fixed plane
  // offsets instead of the select were slower: 10.52 vs 10.04 us at C2; one
  // exec-masked OR on the single mark plane gains nothing either: 9.32 vs
  // 9.15 us.)
  const int delta = (int)(L.fpr - L.negr) * (int)sizeof(WT);
  const uint32_t a = (on && !dup && !premarked) ? (R.P >> 6) : sink_m;
  WT* tgt = reinterpret_cast<WT*>((char*)((lds_char*)(uintptr_t)a + delta));  // free or obstacle: the grid tells
  if (frow_valid) {  // dense: most rays skip; an exec-masked OR of the few that mark
    if (on && !dup && !premarked) lds_or<WT>(tgt, bit);
  } else {
    lds_or<WT>(tgt, bit);
  }
  R.live = on && !hit;
  return on;
}

// --------------------------------------------------------------------------
// Fan march: dense beam sets (lidar.py:34-63).  Every beam belongs to an
// octant class (major axis and sign, minor sign; mc_set_beam_table) and all of
// a class's beams sit on the same line at step k: the row (or column) k cells
// from the robot.  A sector is up to kFanS beams of one class, ordered by
// minor offset, that are never more than one cell apart at any step, so at
// step k its beams cover the cells lo(k) .. lo(k) + 5 of the line and the
// beam -> cell map is the monotone map D(k).  A lane marches one (agent,
// sector) with the live beams A as bits: the cells lit at step k are
// spread[D][A] (each is marked: free up to the first obstacle, and that
// obstacle), and the beams whose cell is an obstacle, expand[D][F], leave A.
// One step is a few bit operations and three LUT / table reads for up to six
// beams, where the ray march spends a dozen VALU operations per ray and step.
// A beam whose step bits depend on the start coordinate (Beam::axis bit 1;
// C4: 270 and 315 degrees, for minor starts 1..3) marches in its sector with
// its common bits unless its robot's start lies in the beam's exceptional
// range; then the sector leaves it out and the lane marches it alone, from
// the start's own bits, after the sectors (a pass only waves with such a
// robot take).  Column lines read and mark the column planes (cneg / cmark /
// cseen), which the stage fills with transposed tiles and gather_marks
// transposes back.  Cells the agent has seen (cseen / fldr) are not marked
// again (dense_beams).
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const lds_char*)(const char*)p;
}
template <typename T>
__device__ __forceinline__ T* lds_ptr(uint32_t a) {
  return reinterpret_cast<T*>((char*)((lds_char*)(uintptr_t)a));
}

#ifndef MC_FAN_SU  // fan_pair's steps per batch (5: C4's 20 steps in 4 batches, 115 VGPRs; 8 needs 144)
#define MC_FAN_SU 5
#endif
// one (agent, sector pair): the two sectors of one line (minor sign + / -),
// entries T[2k], T[2k + 1] of step k (T[0], T[1]: class bits), live beams A0,
// A1.  The line word of step k is read once for both sectors (grid cells and
// seen cells) and their new marks go out as one OR.
template <typename WT, int KM>
__device__ __forceinline__ void fan_pair(const State& s, const Lds<WT>& L, const uint32_t* T, int a,
                                         uint32_t A0, uint32_t A1, int kt) {
  constexpr int SU = MC_FAN_SU;  // steps per batch: reads, then the live-beam chains, then marks
  const uint32_t MD = (uint32_t)(row_plane_words(s.N, s.TW, (int)sizeof(WT)) * (int)sizeof(WT));  // neg -> marks
  const uint8_t* spread = reinterpret_cast<const uint8_t*>(L.fan);
  const uint8_t* expand = spread + 2048;
  const uint32_t desc = T[0];
  const bool cols = (desc & FAN_COLS) != 0;
  const int lx = L.x[a] - 8 * L.bx[a], ly = L.y[a] - 8 * L.by[a];
  // the line's word in the neg plane (row lx + sign k, or column ly + sign k);
  // marks MD bytes on, seen cells 2 MD on
  const uint32_t P0 = lds_addr(cols ? L.cneg : L.negr) + (uint32_t)row_word<WT>(s, a, cols ? ly : lx) * sizeof(WT);
  const int stride = ((desc & FAN_NEG) ? -1 : 1) * row_step<WT>(s) * (int)sizeof(WT);
  const int bb = (cols ? lx : ly) - 32;  // bit of the cell at minor offset lo: bb + (lo + 32)
  const uint2* T2 = reinterpret_cast<const uint2*>(T);
  for (int k0 = 1; k0 <= kt; k0 += SU) {
    uint32_t e0[SU], e1[SU], F0[SU], F1[SU], S0[SU], S1[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      e0[u] = e1[u] = F0[u] = F1[u] = S0[u] = S1[u] = 0;
      if (KM > 0 ? (k0 + u <= KM) : (k0 + u <= kt)) {
        const uint2 e = T2[k0 + u];
        e0[u] = e.x;
        e1[u] = e.y;
        const uint32_t P = P0 + (uint32_t)((k0 + u) * stride);
        const WT fw = *lds_ptr<const WT>(P), sw = *lds_ptr<const WT>(P + 2 * MD);
        const int sh0 = bb + (int)(e0[u] & 63u), sh1 = bb + (int)(e1[u] & 63u);
        F0[u] = (uint32_t)(fw >> sh0) & 63u;
        F1[u] = (uint32_t)(fw >> sh1) & 63u;
        S0[u] = (uint32_t)(sw >> sh0) & 63u;
        S1[u] = (uint32_t)(sw >> sh1) & 63u;
      }
    }
    uint32_t k0v[SU], k1v[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      k0v[u] = expand[(e0[u] & 0x7C0u) | F0[u]];
      k1v[u] = expand[(e1[u] & 0x7C0u) | F1[u]];
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      A0 &= e0[u] >> 16;  // in range (a step past the trip count, or an empty sector, has e = 0)
      A1 &= e1[u] >> 16;
      // (+ for |: the fields are disjoint, A <= 63 -- one v_add3 with the
      // LUT base instead of an OR and an add)
      const uint32_t l0 = spread[(e0[u] & 0x7C0u) + A0], l1 = spread[(e1[u] & 0x7C0u) + A1];
      A0 &= ~k0v[u];
      A1 &= ~k1v[u];
      F0[u] = l0 & ~S0[u];  // new marks (the cells the agent has not seen)
      F1[u] = l1 & ~S1[u];
    }
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      if (F0[u] | F1[u]) {
        const uint32_t P = P0 + (uint32_t)((k0 + u) * stride);
        const WT m = ((WT)F0[u] << (bb + (int)(e0[u] & 63u))) | ((WT)F1[u] << (bb + (int)(e1[u] & 63u)));
        lds_or<WT>(lds_ptr<WT>(P + MD), m);
      }
    }
  }
}

template <int NT, int EPW, typename WT, int KM>
__device__ __forceinline__ void fan_march(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int N = s.N;
  const int kt = KM > 0 ? KM : s.fan_kt;
  const int npair = s.fan_nsec >> 1, nspec = s.fan_nspec;
  const int RW = 2 * (kt + 1);  // words per pair record
  const int qs = N * npair;     // (agent, sector pair) lane items
  const uint32_t* sec = L.fan + kFanLutBytes / 4;
  const uint32_t* sdesc = sec + npair * RW;  // special beams: 8 words each
  // special beam i of (agent, special) pairs: lane (qs + i) % LPE
  // (mc_set_beam_table keeps N * nspec <= lanes per env) loads the start word
  // of its robot's post-move cell now, for the pass after the sectors
  uint32_t spw = 0;
  bool exc = false;
  int si = C.sub - qs % LPE;
  if (si < 0) si += LPE;
  if (nspec > 0 && si < N * nspec) {
    const int a = si / nspec;
    const uint32_t* d = sdesc + 8 * (si - a * nspec);
    const int c0 = (d[1] & FAN_COLS) ? L.x[a] : L.y[a];  // the minor coordinate
    exc = c0 >= (int)d[4] && c0 <= (int)d[5];
    if (exc) spw = (uint32_t)s.beam_bits[(size_t)d[0] * s.bcmax + c0];
  }
  for (int q = C.sub; q < qs; q += LPE) {
    const int pg = q / N, a = q - pg * N;
    const uint32_t* T = sec + pg * RW;
    uint32_t A[2] = {63u, 63u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t desc = T[h];
      if (desc & FAN_SPECIAL) {  // the sector's special beam: left out from an exceptional start
        const uint32_t* d = sdesc + 8 * (desc >> 8);
        const int c0 = (desc & FAN_COLS) ? L.x[a] : L.y[a];
        if (c0 >= (int)d[4] && c0 <= (int)d[5]) A[h] &= ~(1u << ((desc >> 3) & 7u));
      }
    }
    fan_pair<WT, KM>(s, L, T, a, A[0], A[1], kt);
  }
  if (__ballot(exc)) {  // one-beam march of the left-out beams, from the start's bits
    if (exc) {
      const int a = si / nspec;
      const uint32_t* d = sdesc + 8 * (si - a * nspec);
      const int msign = (int)d[2], K = (int)d[3];
      uint32_t* W = L.fspec + si * RW;  // a pair record with an empty second sector
      W[0] = W[1] = d[1];
      int lo = 0;
      for (int k = 1; k <= kt; ++k) {
        lo += ((spw >> (k - 1)) & 1u) ? msign : 0;
        W[2 * k] = (uint32_t)(lo + 32) | (K >= k ? (1u << 16) : 0u);
        W[2 * k + 1] = 0u;
      }
      fan_pair<WT, KM>(s, L, W, a, 1u, 0u, kt);
    }
  }
}

template <int NT, int EPW, typename WT, int SUK, int KN, int KM = 0, int RPLX = 0>
__device__ __forceinline__ void sense(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  constexpr int RPL = RPLX > 0 ? RPLX : Ctx<NT, EPW, WT>::RPL;
  constexpr int SU = SUK;
  const Lds<WT>& L = C.L;
  const int N = s.N, TW = s.TW, TW2 = TW * TW;
  if (s.sensor == 0) {
    // step 0 of every beam is the robot's own (free) cell; with common beam
    // patterns the step-1 cells too (State::beam_k1: every beam reaches its
    // step-1 cell, lidar.py:52-56).  Marked once per agent -- one lane per
    // (agent, row x-1 .. x+1) -- instead of once per ray: at step 1 the rays
    // of an agent crowd three row words, the worst same-address ORs of the
    // march
    const uint32_t k1 = s.beam_k1;
    const int nm = k1 ? 3 * N : N;
    for (int m = C.sub; m < nm; m += LPE) {
      const int a = k1 ? m / 3 : m;
      const int dx = k1 ? m - 3 * a - 1 : 0;
      const uint32_t b3 = k1 ? (k1 >> (3 * (dx + 1))) & 7u : 2u;  // cells y-1, y, y+1
      const int lx = L.x[a] - 8 * L.bx[a] + dx, ly = L.y[a] - 8 * L.by[a] - 1;  // ly >= H >= 1
      if (b3) lds_or<WT>(&L.fpr[row_word<WT>(s, a, lx)], (WT)b3 << ly);
    }
    if (fan_on(s)) {
      fan_march<NT, EPW, WT, KM>(s, C);
      return;
    }
    WT* sink = L.sink + (threadIdx.x & 63);
    const uint32_t sink_m = (uint32_t)(uintptr_t)(const lds_char*)(const char*)sink -
                            (uint32_t)((L.fpr - L.negr) * (int)sizeof(WT));
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
      // lies inside the staged window).  SU steps per batch: the batch's row
      // reads are all issued before its first mark, so no read waits behind
      // an LDS atomic (LDS ops complete in order).
      const int kmax = s.beam_kmax;
      // dense beam sets: adjacent beams share cells for many steps (C4: 360
      // beams, 1 degree apart); sparse ones only next to the robot
      const bool dense = dense_beams(s);
      for (int k0 = 1; k0 <= kmax; k0 += SU) {
        WT nr[SU][RPL], fr[SU][RPL];
        Ray q0[RPL];
#pragma unroll
        for (int j = 0; j < RPL; ++j) q0[j] = q[j];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          if (k0 + u <= kmax) {  // uniform
#pragma unroll
            for (int j = 0; j < RPL; ++j) {
              nr[u][j] = *ray_word<WT>(L, L.negr, q[j]);
              fr[u][j] = dense ? *ray_word<WT>(L, L.fldr, q[j]) : (WT)0;
              ray_advance(q[j], k0 + u);
            }
          }
        }
#pragma unroll
        for (int j = 0; j < RPL; ++j) q[j] = q0[j];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          if (k0 + u <= kmax) {
            bool prev_on = false;
            uint32_t prev_p = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < RPL; ++j) {
              const bool dup = dense && prev_on && q[j].P == prev_p;
              prev_p = q[j].P;
              prev_on = ray_mark<WT, KN>(L, q[j], k0 + u, nr[u][j], fr[u][j], sink_m, dup, dense,
                                         k1 != 0 && k0 + u == 1);
              ray_advance(q[j], k0 + u);
            }
          }
        }
      }
    }
  } else {
    // window [x-r, x+r] x [y-r, y+r] clamped to the padded grid; the
    // reference overwrites it with clip(g,0,1) / clip(-g,0,1), which on a
    // static grid is an OR (every free bit comes from clip(g,0,1)).
    const int rr = s.sq_r;
    for (int idx = C.sub; idx < N * TW2; idx += LPE) {
      const int a = udiv(idx, s.mg_TW2), rem = idx - a * TW2;
      const int ti = udiv(rem, s.mg_TW), tj = rem - ti * TW;
      const int r0 = 8 * (L.bx[a] + ti), c0 = 8 * (L.by[a] + tj);  // tile's first cell
      const int xa = L.x[a], ya = L.y[a];
      const int xlo = max(xa - rr, 0), xhi = min(xa + rr, s.Wp - 1);
      const int ylo = max(ya - rr, 0), yhi = min(ya + rr, s.Lp - 1);
      const uint64_t m = tile_rect(xlo - r0, xhi - r0, ylo - c0, yhi - c0);
      L.fp[idx] = L.pos[idx] & m;
      L.op[idx] = L.neg[idx] & m;
    }
  }
}

// lidar: mark rows -> mark tiles (after the march, before the merge)
// The lane keeps its items' marks in registers for the merge; only the free
// marks go to LDS (other lanes' union dedup reads them).
template <int NT, int EPW, typename WT, int KI>
__device__ __forceinline__ void gather_marks(const State& s, const Ctx<NT, EPW, WT>& C, Items<KI>& I) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int TW = s.TW, TW2 = TW * TW;
  const int items = s.N * TW2;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    I.mf[k] = I.mo[k] = 0;
    if (idx < items) {
      const int a = udiv(idx, s.mg_TW2), rem = idx - a * TW2;
      const int ti = udiv(rem, s.mg_TW), tj = rem - ti * TW;
      uint64_t m = gather_tile<WT>(L.fpr, row_word<WT>(s, a, 8 * ti), row_step<WT>(s), tj);
      if (fan_on(s))  // the fan's column-line marks, transposed back
        m |= transpose8(gather_tile<WT>(L.cmark, row_word<WT>(s, a, 8 * tj), row_step<WT>(s), ti));
      I.mf[k] = m & ~I.n[k];
      I.mo[k] = m & I.n[k];
      L.fp[idx] = I.mf[k];
    }
  }
}

// single_square_tool: only the robot's own cell becomes free (:233-234)
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void single_tool(const State& s, const Ctx<NT, EPW, WT>& C) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int TW = s.TW, TW2 = TW * TW;
  for (int idx = C.sub; idx < s.N * TW2; idx += LPE) {
    const int a = udiv(idx, s.mg_TW2);
    const int lx = L.x[a] - 8 * L.bx[a], ly = L.y[a] - 8 * L.by[a];
    const int own = (a * TW + (lx >> 3)) * TW + (ly >> 3);
    L.fp[idx] = (own == idx) ? (1ull << tile_bit(lx, ly)) : 0ull;
  }
}

// --------------------------------------------------------------------------
// merge (dec_grid_rl.py:232-256): newly set free bits per agent, and the
// union delta = cells some agent marked this step that were not yet visited,
// each counted at the lowest-index agent that marked it.  Agents' blocks are
// aligned to the global tile grid: the same map tile is the same word in
// every block that holds it.  Also folds the marks into the old tiles (the
// obs crops read the post-step maps).
// --------------------------------------------------------------------------
// marks_in_regs: the lidar's free marks are in I.mf (else L.fp: the square
// sensor, or single_square_tool's own cell); obst_in_regs: its obstacle marks
// are in I.mo (lidar, with or without single_square_tool; else L.op)
template <int NT, int EPW, typename WT, int KI, int NS>
__device__ __forceinline__ void merge(const State& s, const Ctx<NT, EPW, WT>& C, Items<KI>& I,
                                      bool marks_in_regs, bool obst_in_regs) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int TW = s.TW;
  const int items = s.N * TW * TW;
  // compile-time agent count: every lower agent's block origin once, in
  // registers (broadcast LDS reads issued together)
  int BX[NS > 0 ? NS : 1], BY[NS > 0 ? NS : 1];
  if constexpr (NS > 0) {
#pragma unroll
    for (int b = 0; b < NS; ++b) {
      BX[b] = L.bx[b];
      BY[b] = L.by[b];
    }
  }
  // EPW == 1: agent j's block origin in lane j of every wave, broadcast by
  // v_readlane (N <= 64)
  const int jw = (int)(threadIdx.x & 63);
  const int jl = jw < s.N ? jw : 0;
  const int abx = L.bx[jl], aby = L.by[jl];
  // EPW == 1 without a compile-time agent count <= 8 (C5: 16 agents):
  // lane j (< N) of every wave holds ovj, bit b = a lower-index agent b whose
  // block overlaps agent j's; an item fetches its agent's mask from lane a
  // (ds_bpermute) and reads only those agents' marks -- usually none, where
  // the loop over every lower agent ran up to N - 1 readlane rounds per item
  uint64_t ovj = 0;
  if constexpr (NS == 0 && EPW == 1 && MC_ABL != 3) {
    // branch-free: |dx| < TW as one unsigned compare, the b < j condition as
    // one mask at the end (per-b lane conditions became exec-mask branches
    // with spilled SGPR masks)
    const uint32_t span = (uint32_t)(2 * TW - 1);
    uint32_t lo = 0, hi = 0;
    for (int b = 0; b < s.N - 1; ++b) {  // uniform trip count (unrolled when N is compiled in)
      const int bxb = rdlane(abx, b), byb = rdlane(aby, b);
      const uint32_t ov = (uint32_t)((uint32_t)(abx - bxb + TW - 1) < span) & (uint32_t)((uint32_t)(aby - byb + TW - 1) < span);
      if (b < 32) lo |= ov << b;
      else hi |= ov << (b - 32);
    }
    ovj = ((uint64_t)hi << 32 | lo) & (jw >= 64 ? ~0ull : ((1ull << jw) - 1ull));
  }
  // (fetched with every lane active: ds_bpermute reads 0 from inactive lanes)
  uint64_t ova[KI];
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    ova[k] = 0;
    if constexpr (NS == 0 && EPW == 1) {
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)ovj, I.a[k]);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(ovj >> 32), I.a[k]);
      ova[k] = (uint64_t)lo | ((uint64_t)hi << 32);
    }
  }
  uint32_t cf = 0, cv = 0;
#ifdef MC_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(14);  // the staged mask tiles landed
#endif
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    const int idx = C.sub + k * LPE;
    I.nf[k] = I.no[k] = I.nu[k] = 0;
    if (idx < items) {
      const uint64_t fp = marks_in_regs ? I.mf[k] : L.fp[idx];
      const uint64_t op = obst_in_regs ? I.mo[k] : L.op[idx];
      uint64_t f0, o0, u0;
      old_tiles<KI>(I, k, f0, o0, u0);  // first use of the mask loads
      I.f[k] = f0;
      I.o[k] = o0;
      I.nf[k] = fp & ~f0;
      I.no[k] = op & ~o0;
      L.fold[idx] = f0 | fp;
      L.oold[idx] = o0 | op;
      if (s.dist && MC_ABL != 2) {
        // dist_reward: the post-step free tile's 8 rows into the (dead)
        // mark-row plane, for dist_window (byte tj of block rows 8 ti ..)
        uint8_t* rb = reinterpret_cast<uint8_t*>(L.fpr);
        const size_t off = (size_t)row_word<WT>(s, I.a[k], 8 * I.ti[k]) * sizeof(WT) + I.tj[k];
        const size_t rs = (size_t)row_step<WT>(s) * sizeof(WT);
        const uint64_t ft = f0 | fp;
#pragma unroll
        for (int r = 0; r < 8; ++r) rb[off + r * rs] = (uint8_t)(ft >> (8 * r));
      }
      cf += __popcll(I.nf[k]);
      uint64_t cand = fp & ~u0;
      const int a = I.a[k], gi = I.gi[k], gj = I.gj[k];
      if constexpr (NS > 0) {
        // marks of lower-index agents in this tile: every read issued
        // unconditionally (own tile when unused), no loop-carried branch
        // (an agent whose block misses the tile, or b >= a, reads the
        // slot's zero word)
        uint64_t t[NS > 1 ? NS - 1 : 1];
#pragma unroll
        for (int b = 0; b < NS - 1; ++b) {
          const int bi = gi - BX[b], bj = gj - BY[b];
          const bool use = b < a && (unsigned)bi < (unsigned)TW && (unsigned)bj < (unsigned)TW;
          t[b] = *(use ? &L.fp[(b * TW + bi) * TW + bj] : &L.sc->zero);
        }
#pragma unroll
        for (int b = 0; b < NS - 1; ++b) cand &= ~t[b];
      } else if constexpr (EPW == 1) {
        for (uint64_t m = ova[k]; m; m &= m - 1ull) {
          const int b = __ffsll((unsigned long long)m) - 1;
          const int bi = gi - L.bx[b], bj = gj - L.by[b];
          if ((unsigned)bi < (unsigned)TW && (unsigned)bj < (unsigned)TW)
            cand &= ~L.fp[(b * TW + bi) * TW + bj];
        }
      } else {
      for (int b = 0; b < s.N - 1; ++b) {
        if (b >= a) break;
        const int bi = gi - L.bx[b], bj = gj - L.by[b];
        if ((unsigned)bi < (unsigned)TW && (unsigned)bj < (unsigned)TW)
          cand &= ~L.fp[(b * TW + bi) * TW + bj];
      }
      }
      I.nu[k] = cand;
      cv += __popcll(cand);
      // dist_reward: a new free cell closer than M to the agent's witness
      // may lower max(d): the map's M must be recomputed (mc_dist.hip)
      if (s.dist && I.nf[k]) {
        const int M = L.dm[a], w = L.dw[a];
        if (M > 0 && bits_within(I.nf[k], 8 * gi, 8 * gj, witness_x(w), witness_y(w), M))
          atomicOr((unsigned long long*)&L.sc->dist_hit, 1ull << a);
      }
    }
  }
  if (cf) atomicAdd(&L.sc->cnt_free, cf);
  if (cv) atomicAdd(&L.sc->cnt_vis, cv);
}

// dist_reward POST terms (dec_grid_rl.py:222-223,239-240,260-282,350-352)
// of the agents whose max(d) M is still known (mc_dist.hip): d of each target
// -- the 5 end cells of the next step at the quirk index (padded-grid x, y
// read without the pad offset) and the E x E crop -- is the L1 distance to
// the nearest covered cell of the agent's staged block (post-step free rows,
// written into fpr by merge), exact when it does not exceed b, the distance
// from the target to the nearest cell outside the block (any covered cell
// there is at least b away).  Rows are scanned outward from the target's row
// until the row distance reaches the best d.  Writes pre[e][a] (M, d of the
// end cells) and the float obs crop; an agent with a target it cannot settle
// is flagged in dist_fail (listed for the full transform, which rewrites its
// terms).  `skip`: agents left to the full transform anyway (as is every
// agent whose M is unknown).
template <typename WT>
__device__ __forceinline__ int row_dist(WT row, int c) {  // |c - nearest set bit|, or a large value
  const WT lo = row & (((WT)2 << c) - (WT)1), hi = row >> c;
  int h = 1 << 20;
  if constexpr (sizeof(WT) == 4) {
    if (lo) h = c - (31 - __clz((uint32_t)lo));
    if (hi) h = min(h, __ffs((uint32_t)hi) - 1);
  } else {
    if (lo) h = c - (63 - __clzll((unsigned long long)lo));
    if (hi) h = min(h, __ffsll((unsigned long long)hi) - 1);
  }
  return h;
}

template <int NT, int EPW, typename WT>
__device__ __forceinline__ void dist_window(const State& s, const Ctx<NT, EPW, WT>& C, uint64_t skip) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int N = s.N, E = s.E, T = 5 + E * E, RB = 8 * s.TW;
  const WT cols = sizeof(WT) == 8 && RB >= 64 ? ~(WT)0 : (WT)(((uint64_t)1 << RB) - 1);  // the block's columns
  float* pre = const_cast<float*>(s.dist_pre);
  for (int idx = C.sub; idx < N * T; idx += LPE) {
    const int a = idx / T, t = idx - a * T;
    const int M = L.dm[a];
    if (((skip >> a) & 1ull) || M < 0) continue;
    const int px = L.x[a], py = L.y[a];
    int tx, ty;
    if (t < 5) {
      tx = px + (t == 1 ? 1 : (t == 3 ? -1 : 0)) - s.pad;
      ty = py + (t == 2 ? 1 : (t == 4 ? -1 : 0)) - s.pad;
    } else {
      const int k = t - 5, r = k / E;
      tx = px - s.ego + r;
      ty = py - s.ego + (k - r * E);
    }
    const int lx = tx - 8 * L.bx[a], ly = ty - 8 * L.by[a];
    const int b = min(min(lx, RB - 1 - lx), min(ly, RB - 1 - ly)) + 1;  // <= 0: outside the block
    int d = b + 1;
    if (b > 0) {
      // the target's row, then rows outward while they can help (a covered
      // target, d = 0, is the common case next to the robot: one read)
      d = min(d, row_dist<WT>(L.fpr[row_word<WT>(s, a, lx)] & cols, ly));
      for (int dr = 1; dr < d; ++dr) {
        if (lx - dr >= 0) d = min(d, dr + row_dist<WT>(L.fpr[row_word<WT>(s, a, lx - dr)] & cols, ly));
        if (lx + dr < RB) d = min(d, dr + row_dist<WT>(L.fpr[row_word<WT>(s, a, lx + dr)] & cols, ly));
      }
    }
    if (d > b) {
      atomicOr((unsigned long long*)&L.sc->dist_fail, 1ull << a);
      continue;
    }
    const size_t ea = (size_t)C.e * N + a;
    if (t < 5) pre[ea * 8 + 1 + t] = (float)d;
    else s.dist_obs_out[ea * E * E + (t - 5)] = dist_value((float)d, (float)M);
    if (t == 0) pre[ea * 8] = (float)M;
  }
}

#ifndef MC_DIST_AM  // build knob (A/B): 0 keeps the (agent, target) item loop for T <= 32
#define MC_DIST_AM 1
#endif
// The same terms, agent-major, when the targets fit 32 lanes (T = 5 + E*E
// <= 32, e.g. egoradius 2): lane l of the slot takes target l % 32 of agent
// a0 + l / 32 in pass a0, so a lane's target offsets are computed once for
// every pass (no per-item division into (agent, target) and (row, column)),
// and an agent's skip / M test is uniform over its 32 lanes.
template <int NT, int EPW, typename WT>
__device__ __forceinline__ void dist_window_am(const State& s, const Ctx<NT, EPW, WT>& C, uint64_t skip) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  constexpr int APP = LPE / 32;  // agents per pass
  const Lds<WT>& L = C.L;
  const int N = s.N, E = s.E, T = 5 + E * E, RB = 8 * s.TW;
  const WT cols = sizeof(WT) == 8 && RB >= 64 ? ~(WT)0 : (WT)(((uint64_t)1 << RB) - 1);  // the block's columns
  const int t = C.sub & 31;
  if (t >= T) return;
  // target - robot: the end cells of the next step at the quirk index, the crop
  int ox, oy;
  if (t < 5) {
    ox = (t == 1 ? 1 : (t == 3 ? -1 : 0)) - s.pad;
    oy = (t == 2 ? 1 : (t == 4 ? -1 : 0)) - s.pad;
  } else {
    const int k = t - 5, r = k / E;
    ox = r - s.ego;
    oy = k - r * E - s.ego;
  }
  float* pre_e = const_cast<float*>(s.dist_pre) + (size_t)C.e * N * 8;
  float* obs_e = s.dist_obs_out + (size_t)C.e * N * E * E;
  for (int a0 = 0; a0 < N; a0 += APP) {
    const int a = a0 + (C.sub >> 5);
    if (a >= N) break;
    const int M = L.dm[a];
    if (((skip >> a) & 1ull) || M < 0) continue;
    const int lx = L.x[a] + ox - 8 * L.bx[a], ly = L.y[a] + oy - 8 * L.by[a];
    const int b = min(min(lx, RB - 1 - lx), min(ly, RB - 1 - ly)) + 1;  // <= 0: outside the block
    int d = b + 1;
    if (b > 0) {
      d = min(d, row_dist<WT>(L.fpr[row_word<WT>(s, a, lx)] & cols, ly));
      for (int dr = 1; dr < d; ++dr) {
        if (lx - dr >= 0) d = min(d, dr + row_dist<WT>(L.fpr[row_word<WT>(s, a, lx - dr)] & cols, ly));
        if (lx + dr < RB) d = min(d, dr + row_dist<WT>(L.fpr[row_word<WT>(s, a, lx + dr)] & cols, ly));
      }
    }
    if (d > b) {
      atomicOr((unsigned long long*)&L.sc->dist_fail, 1ull << a);
      continue;
    }
    if (t < 5) pre_e[a * 8 + 1 + t] = (float)d;
    else obs_e[a * E * E + (t - 5)] = dist_value((float)d, (float)M);
    if (t == 0) pre_e[a * 8] = (float)M;
  }
}

#ifndef MC_DIST_AM2  // build knob (A/B): 0 keeps dist_window_am's pass-by-pass loop
#define MC_DIST_AM2 1
#endif
// dist_window_am with the agent count known at compile time (NS): the passes'
// first row reads (the target's own row: the common answer) are issued
// together, then the few lanes whose target is not covered scan outward,
// then the stores -- one LDS latency chain for all passes instead of one per
// pass
template <int NT, int EPW, typename WT, int NS>
__device__ __forceinline__ void dist_window_am2(const State& s, const Ctx<NT, EPW, WT>& C, uint64_t skip) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  constexpr int APP = LPE / 32;               // agents per pass
  constexpr int NP = (NS + APP - 1) / APP;    // passes
  const Lds<WT>& L = C.L;
  const int E = s.E, T = 5 + E * E, RB = 8 * s.TW;
  const WT cols = sizeof(WT) == 8 && RB >= 64 ? ~(WT)0 : (WT)(((uint64_t)1 << RB) - 1);
  const int t = C.sub & 31;
  if (t >= T) return;
  int ox, oy;
  if (t < 5) {
    ox = (t == 1 ? 1 : (t == 3 ? -1 : 0)) - s.pad;
    oy = (t == 2 ? 1 : (t == 4 ? -1 : 0)) - s.pad;
  } else {
    const int k = t - 5, r = k / E;
    ox = r - s.ego;
    oy = k - r * E - s.ego;
  }
  int lxv[NP], lyv[NP], bv[NP], dv[NP], Mv[NP];
  bool on[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int a = p * APP + (C.sub >> 5);
    const int M = L.dm[a < NS ? a : 0];
    on[p] = a < NS && !((skip >> a) & 1ull) && M >= 0;
    Mv[p] = M;
    const int lx = L.x[a < NS ? a : 0] + ox - 8 * L.bx[a < NS ? a : 0];
    const int ly = L.y[a < NS ? a : 0] + oy - 8 * L.by[a < NS ? a : 0];
    lxv[p] = lx;
    lyv[p] = ly;
    bv[p] = min(min(lx, RB - 1 - lx), min(ly, RB - 1 - ly)) + 1;  // <= 0: outside the block
    dv[p] = bv[p] + 1;
    if (on[p] && bv[p] > 0) dv[p] = min(dv[p], row_dist<WT>(L.fpr[row_word<WT>(s, a, lx)] & cols, ly));
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int a = p * APP + (C.sub >> 5);
    if (on[p] && bv[p] > 0) {
      const int lx = lxv[p], ly = lyv[p];
      int d = dv[p];
      for (int dr = 1; dr < d; ++dr) {
        if (lx - dr >= 0) d = min(d, dr + row_dist<WT>(L.fpr[row_word<WT>(s, a, lx - dr)] & cols, ly));
        if (lx + dr < RB) d = min(d, dr + row_dist<WT>(L.fpr[row_word<WT>(s, a, lx + dr)] & cols, ly));
      }
      dv[p] = d;
    }
  }
  float* pre_e = const_cast<float*>(s.dist_pre) + (size_t)C.e * NS * 8;
  float* obs_e = s.dist_obs_out + (size_t)C.e * NS * E * E;
  uint64_t fail = 0;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int a = p * APP + (C.sub >> 5);
    if (!on[p]) continue;
    if (dv[p] > bv[p]) {
      fail |= 1ull << a;
      continue;
    }
    if (t < 5) pre_e[a * 8 + 1 + t] = (float)dv[p];
    else obs_e[a * E * E + (t - 5)] = dist_value((float)dv[p], (float)Mv[p]);
    if (t == 0) pre_e[a * 8] = (float)Mv[p];
  }
  if (fail) atomicOr((unsigned long long*)&L.sc->dist_fail, fail);
}

template <bool O32>
__device__ __forceinline__ void st_tile(uint64_t* base, uint32_t idx, uint64_t v) {
  if constexpr (O32) *reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(base) + (size_t)(idx << 3)) = v;
  else base[idx] = v;
}

template <int NT, int EPW, typename WT, int KI, bool O32 = false>
__device__ __forceinline__ void store_tiles(const State& s, const Ctx<NT, EPW, WT>& C,
                                            const Items<KI>& I) {
  const uint32_t mt = (uint32_t)s.MT;
#pragma unroll
  for (int k = 0; k < KI; ++k) {
    if (!I.in[k]) continue;
    const uint32_t gt = tile_index24(s.TCS, I.gi[k], I.gj[k]);
    const uint32_t fb = __umul24((uint32_t)C.e * (uint32_t)s.N + (uint32_t)I.a[k], mt) + gt;
    // only obstacle marks can fall on an edge tile's cells beyond the map
    const uint64_t no = I.no[k] & tile_in_grid(s, I.gi[k], I.gj[k]);
    if (I.nf[k]) st_tile<O32>(s.freem, fb, I.f[k] | I.nf[k]);  // one writer per agent tile
    if (no) st_tile<O32>(s.obstm, fb, I.o[k] | no);
    if (I.nu[k]) {  // agents' blocks overlap: several lanes may add bits to one tile
      const uint32_t vb = (__umul24((uint32_t)C.e, mt) + gt) << 3;
      unsigned long long* vp = O32 ? reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(s.vis) + (size_t)vb)
                                   : (unsigned long long*)(s.vis + (__umul24((uint32_t)C.e, mt) + gt));
      atomicOr(vp, I.nu[k]);
    }
  }
}

#ifndef MC_RELOAD  // build knob (A/B): 0 keeps one State for the whole kernel
#define MC_RELOAD 1
#endif
// The kernel's State re-read at a phase boundary from the kernel arguments
// through an opaque kernarg pointer: the fields the next phase uses are
// loaded there (s_load, scalar cache) instead of staying live in SGPRs across
// the whole kernel, where the C5 shape's ~35 pointers spilled to VGPR lanes
// (v_writelane at entry, a VALU v_readlane at every use).  One env per
// workgroup only: the two-env C2 wave spilled more with it and ran slower
// (8.38 vs 8.22 us; C4 126.6 -> 123.3 us, C5 steady 140.7 -> 136.4 us per
// step, profiles/r6/rlab/)
// The env kernel's one argument: the State and the step's buffers
struct EnvIO {
  const uint8_t* actions;   // [B][N] (MODE_STEP)
  const uint8_t* env_mask;  // [B] envs to reset (MODE_RESET; null: all)
  const int32_t* inj_pos;   // [B][N][2] injected start cells (null: device draw)
  double* reward_out;
  uint8_t* done_out;
  uint8_t* obs_out;
  uint8_t* adj_out;  // null: no comm graph output
  int mode;
};
struct EnvArgs {
  State s;
  EnvIO io;
};
template <class SH, int EPW>
__device__ __forceinline__ void reload_state(State& s, EnvIO& io) {
  if constexpr (MC_RELOAD != 0 && EPW == 1) {
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();  // the EnvArgs
    asm volatile("" : "+s"(kp));
    const EnvArgs& A = *(const EnvArgs*)kp;
    s = A.s;
    io = A.io;
    specialize<SH>(s);
  }
}
template <class SH, int EPW>
__device__ __forceinline__ void reload_state(State& s) {
  EnvIO io;
  reload_state<SH, EPW>(s, io);
}
// (also inside sense_and_merge / reset_env: slower, C4 123.9 vs 123.2 us, C5
// steady 137.0 vs 136.3 us, profiles/r6/rlab2/)
#ifndef MC_RELOAD_INNER  // build knob (A/B): 1 = re-read inside sense_and_merge / reset_env too
#define MC_RELOAD_INNER 0
#endif
#ifndef MC_UNIFORM_FLAGS  // build knob (A/B): 0 keeps the env flags as lane values
#define MC_UNIFORM_FLAGS 1
#endif
template <class SH, int EPW>
struct Reload {
  __device__ __forceinline__ void operator()(State& s) const {
    if constexpr (MC_RELOAD_INNER != 0) reload_state<SH, EPW>(s);
  }
};
struct NoReload {
  __device__ __forceinline__ void operator()(State&) const {}
};

// sense -> (lidar: gather) -> (single tool) -> merge, with the barriers (rl:
// the State re-read between them, reload_state)
template <int NT, int EPW, typename WT, int KI, int SUK, int NS, int KN, int KM = 0, int RPLX = 0,
          class RL = NoReload>
__device__ __forceinline__ void sense_and_merge(const State& s0, const Ctx<NT, EPW, WT>& C,
                                                Items<KI>& I, RL rl = RL()) {
  State s = s0;
  if (MC_ABL != 5) sense<NT, EPW, WT, SUK, KN, KM, RPLX>(s, C);
  __syncthreads();
  STAMP(13);
  rl(s);
  if (s.sensor == 0) {
    gather_marks<NT, EPW, WT, KI>(s, C, I);
    __syncthreads();
  }
  STAMP(4);
  rl(s);
  if (s.sst) {
    single_tool<NT, EPW, WT>(s, C);
    __syncthreads();
  }
  merge<NT, EPW, WT, KI, NS>(s, C, I, s.sensor == 0 && !s.sst, s.sensor == 0);
}

// --------------------------------------------------------------------------
// reset (dec_grid_rl.py:449-531) of the slot's env inside the launch: grid
// pick, start cells (injected, or Philox rejection draw with the reference's
// acceptance rule, :491-502), zeroed maps, initial observe() (reward
// discarded, :524).
// --------------------------------------------------------------------------
template <typename WT>
__device__ __forceinline__ void set_agent(const State& s, const Lds<WT>& L, int a, int x, int y) {
  L.x0[a] = L.x[a] = x;
  L.y0[a] = L.y[a] = y;
  L.bx[a] = (x - s.H - 1) >> 3;  // arithmetic shift: floor for negatives
  L.by[a] = (y - s.H - 1) >> 3;
}

template <int NT, int EPW, typename WT, int SUK, int NS, int KN, bool O32, int KM = 0, int RPLX = 0,
          class RL = NoReload>
__device__ __forceinline__ void reset_env(const State& s, const Ctx<NT, EPW, WT>& C,
                                          const int32_t* inj_pos, RL rl = RL()) {
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
      const uint4 r = philox(s.seed, make_uint4(0xFFFFFFFFu, s.env0 + (uint32_t)e, ep, 0x67726964u));
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
  const size_t mt = (size_t)s.MT;
  {  // zero this env's maps (:505-514)
    uint64_t* f = s.freem + (size_t)e * N * mt;
    uint64_t* o = s.obstm + (size_t)e * N * mt;
    for (size_t i = C.sub; i < (size_t)N * mt; i += LPE) { f[i] = 0; o[i] = 0; }
    uint64_t* v = s.vis + (size_t)e * mt;
    for (size_t i = C.sub; i < mt; i += LPE) v[i] = 0;
  }
  if (inj_pos != nullptr) {
    if (C.sub < N) {
      const int x = inj_pos[((size_t)e * N + C.sub) * 2];
      const int y = inj_pos[((size_t)e * N + C.sub) * 2 + 1];
      bool bad = grid_blocked(s, g, x, y);
      for (int j = 0; j < C.sub; ++j)
        bad |= (inj_pos[((size_t)e * N + j) * 2] == x && inj_pos[((size_t)e * N + j) * 2 + 1] == y);
      if (bad) atomicOr(s.err, ERR_INJECT);
      set_agent<WT>(s, L, C.sub, x, y);
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
      const uint4 r = philox(s.seed, make_uint4(k, s.env0 + (uint32_t)e, ep, 0x706c6163u));
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
    if (lane < N) set_agent<WT>(s, L, lane, px, py);
  }
  // the zeroing stores must land before the window stores / atomics below
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  Items<KI> I;
  zero_marks<NT, EPW, WT>(s, C);
  stage<NT, EPW, WT, KI, O32>(s, C, g, /*load_masks=*/false, I);
  __syncthreads();
  sense_and_merge<NT, EPW, WT, KI, SUK, NS, KN, KM, RPLX>(s, C, I, rl);
  store_tiles<NT, EPW, WT, KI, O32>(s, C, I);
  __syncthreads();
  if (C.sub == 0) {
    s.free_cnt[e] = L.sc->cnt_free;
    s.vis_cnt[e] = L.sc->cnt_vis;
    s.currstep[e] = 0;
  }
}

// --------------------------------------------------------------------------
// obs (dec_grid_rl.py:312-372): layer 0 robot_pad, 1 own free, 2 own obst,
// E x E around each robot, uint8 [N][Lc][E][E] per env.  A lane builds four
// consecutive E-bit crop rows in registers: their 4E bytes are exactly E
// dwords of the output (each dword = 4 bits spread to bytes by a multiply).
// --------------------------------------------------------------------------
// Robot cells for the robot_pad layer: registers when the agent count is a
// compile-time constant NS <= 8, LDS otherwise.
template <int NS>
struct Robots {
  int x[NS > 0 ? NS : 1], y[NS > 0 ? NS : 1];
};

template <typename WT, int NS>
__device__ __forceinline__ uint64_t obs_row(const State& s, const Lds<WT>& L, const Robots<NS>& R,
                                            uint64_t moved, int row) {
  const int E = s.E, ego = s.ego, Lc = s.Lc, TW = s.TW;
  const int a = udiv(row, s.mg_LcE), rem = row - a * (Lc * E);
  const int layer = udiv(rem, s.mg_E), r = rem - layer * E;
  const int xa = L.x[a], ya = L.y[a];
  if (layer == 0) {
    const int cx = xa - ego + r, cy0 = ya - ego;
    uint64_t bits = 0;
    if constexpr (NS > 0) {
#pragma unroll
      for (int j = 0; j < NS; ++j) {
        const int dc = R.y[j] - cy0;
        const bool on = ((moved >> j) & 1) && R.x[j] == cx && dc >= 0 && dc < E;
        bits |= on ? (1ull << dc) : 0ull;
      }
    } else {
      for (uint64_t m = moved; m; m &= m - 1) {
        const int j = __ffsll((unsigned long long)m) - 1;
        const int dc = L.y[j] - cy0;
        if (L.x[j] == cx && dc >= 0 && dc < E) bits |= 1ull << dc;
      }
    }
    return bits;
  }
  if (layer > 2) return 0;  // dijkstra layer: written by mc_dijkstra.hip
  // layers 1, 2: crop row = bits [ly0, ly0+E) of block row lx, gathered from
  // the row's byte in consecutive tiles of the block
  const int lx = xa - ego + r - 8 * L.bx[a];
  const int ly0 = ya - ego - 8 * L.by[a];
  const uint64_t* plane = layer == 1 ? L.fold : L.oold;
  const int t0 = (a * TW + (lx >> 3)) * TW + (ly0 >> 3);
  const int sh = (lx & 7) * 8;
  uint64_t acc;
  if (E <= 9) {  // at most two tiles; a second byte past the crop is masked off
    acc = ((plane[t0] >> sh) & 0xFFull) | (((plane[t0 + 1] >> sh) & 0xFFull) << 8);
  } else {
    const int nt = ((ly0 & 7) + E + 7) >> 3;
    acc = 0;
    for (int q = 0; q < nt; ++q) acc |= ((plane[t0 + q] >> sh) & 0xFFull) << (8 * q);
  }
  return (acc >> (ly0 & 7)) & low_mask(E);
}

template <int NT, int EPW, typename WT, int NS>
__device__ __forceinline__ void write_obs(const State& s, const Ctx<NT, EPW, WT>& C,
                                          uint8_t* obs_out) {
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  const Lds<WT>& L = C.L;
  const int E = s.E;
  const int rows = s.N * s.Lc * E;
  const uint64_t moved = L.sc->moved;
  Robots<NS> R;
  if constexpr (NS > 0) {
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      R.x[j] = L.x[j];
      R.y[j] = L.y[j];
    }
  }
  uint8_t* dst = obs_out + (size_t)C.e * rows * E;
  // every env's obs 4-byte aligned and a whole number of 4-row groups
  const bool dwords = E <= 16 && ((rows * E) & 3) == 0 && (rows & 3) == 0;
  if (dwords) {
    // lane q builds rows 2q, 2q+1; lanes 2m, 2m+1 swap them, so each holds the
    // 4-row group m (4E bytes = E dwords) and writes half of its dwords
    for (int q = C.sub; 2 * q < rows; q += LPE) {
      const uint32_t two = (uint32_t)obs_row<WT, NS>(s, L, R, moved, 2 * q) |
                           ((uint32_t)obs_row<WT, NS>(s, L, R, moved, 2 * q + 1) << E);
      const uint32_t other = (uint32_t)__shfl_xor((int)two, 1);
      const bool hi = q & 1;
      const uint64_t cat = hi ? ((uint64_t)other | ((uint64_t)two << (2 * E)))
                              : ((uint64_t)two | ((uint64_t)other << (2 * E)));
      uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + (size_t)(2 * (q & ~1)) * E);
      const int half = (E + 1) >> 1;
      for (int d = hi ? half : 0; d < (hi ? E : half); ++d)
        d32[d] = ((uint32_t)(cat >> (4 * d)) & 0xFu) * 0x00204081u & 0x01010101u;
    }
  } else {
    for (int i = C.sub; i < rows; i += LPE) {
      const uint64_t bits = obs_row<WT, NS>(s, L, R, moved, i);
      for (int c = 0; c < E; ++c) dst[(size_t)i * E + c] = (uint8_t)((bits >> c) & 1u);
    }
  }
}

// Compile-time obs shape (LC = 3 layers, or 4 with the dijkstra layer, which
// is written here as zeros and then by mc_dijkstra.hip; E*E <= 28 bits, whole
// dwords per env): lane j < LC*N of a slot builds the E*E-bit crop of block
// j = (agent j / LC, layer j % LC) -- layer 0 from the robot cells, layers 1
// and 2 from one LDS
// byte per crop row and tile (the crop's bytes in the post-step tiles).  The
// wave's envs are consecutive, so their obs are one run of dwords: lane l
// writes dwords l, l + 64, ...; dword d is the nibble at bit 4d of the
// slot's crop stream (fetched from the crop lanes by ds_bpermute), spread to
// bytes by one multiply.  No per-row or per-layer branches.
template <int EGO, int NS, int LC = 3>
struct ObsFast {
  static constexpr int E = 2 * EGO + 1, EE = E * E, NB = LC * NS;
  static constexpr bool ok = EGO > 0 && NS > 0 && EE <= 28 && (NB * EE) % 4 == 0 &&
                             (LC == 3 || LC == 4);
};

template <int NT, int EPW, typename WT, int NS, int EGO, int LC = 3>
__device__ __forceinline__ void write_obs_fast(const State& s, const Ctx<NT, EPW, WT>& C,
                                               uint8_t* obs_out) {
  using OF = ObsFast<EGO, NS, LC>;
  constexpr int LPE = Ctx<NT, EPW, WT>::LPE;
  constexpr int E = OF::E, EE = OF::EE, NB = OF::NB;
  static_assert(NB <= LPE && NB <= 64, "one crop per lane of the first wave");
  static_assert(NT == 64 || EPW == 1, "one wave, or one env per workgroup");
  const Lds<WT>& L = C.L;
  const int TW = s.TW;
  // ---- crops
  const int j = C.sub < NB ? C.sub : 0;
  const int a = LC == 3 ? (j * 86) >> 8 : j >> 2;  // j / LC for j < 128
  const int layer = j - LC * a;
  const int xa = L.x[a], ya = L.y[a];
  const uint64_t moved = L.sc->moved;
  uint32_t rp = 0;  // layer 0: robot_pad crop (robots that moved since the reset)
#pragma unroll
  for (int i = 0; i < NS; ++i) {
    const int dx = L.x[i] - xa + EGO, dy = L.y[i] - ya + EGO;
    const bool on = ((moved >> i) & 1) && (unsigned)dx < (unsigned)E && (unsigned)dy < (unsigned)E;
    rp |= on ? (1u << (dx * E + dy)) : 0u;
  }
  // layers 1, 2: crop row r = bits [ly0 & 7, +E) of bytes (lx & 7) of tiles
  // (lx >> 3, ly0 >> 3) and the next tile column
  const uint8_t* plane = reinterpret_cast<const uint8_t*>(layer == 2 ? L.oold : L.fold);
  const int lx0 = xa - EGO - 8 * L.bx[a], ly0 = ya - EGO - 8 * L.by[a];
  const uint8_t* t0 = plane + ((size_t)(a * TW) * TW + (ly0 >> 3)) * 8;
  uint32_t fo = 0;
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const int lx = lx0 + r;
    const uint8_t* p = t0 + (size_t)(lx >> 3) * TW * 8 + (lx & 7);
    const uint32_t w = (uint32_t)p[0] | ((uint32_t)p[8] << 8);
    fo |= ((w >> (ly0 & 7)) & ((1u << E) - 1u)) << (r * E);
  }
  const uint32_t crop = layer == 0 ? rp : (layer <= 2 ? fo : 0u);  // layer 3: dijkstra / dist (float buffer)
  if constexpr (NT > 64) {
    // one env per multi-wave workgroup (C4, C5): the first wave's crops go
    // through LDS (the march's dead sink row) to every lane; lane l writes
    // bits [16 l, 16 l + 16) of the env's crop stream as one dwordx4 (16
    // bits span at most two crops: EE >= 16), else dword by dword
    uint32_t* cl = reinterpret_cast<uint32_t*>(L.sink);
    if (C.sub < NB) cl[C.sub] = crop;
    __syncthreads();
    constexpr int DPE = NB * EE / 4;
    uint32_t* out = reinterpret_cast<uint32_t*>(obs_out + (size_t)C.e * (NB * EE));
    if constexpr (DPE % 4 == 0 && EE >= 16) {
      for (int q = C.sub; q < DPE / 4; q += NT) {
        const int i = 16 * q, jb = i / EE, o = i - jb * EE;
        const uint64_t w = (uint64_t)cl[jb] | ((uint64_t)(jb + 1 < NB ? cl[jb + 1] : 0u) << EE);
        const uint32_t bits = (uint32_t)(w >> o);
        uint4 v;
        v.x = ((bits & 0xFu) * 0x00204081u) & 0x01010101u;
        v.y = (((bits >> 4) & 0xFu) * 0x00204081u) & 0x01010101u;
        v.z = (((bits >> 8) & 0xFu) * 0x00204081u) & 0x01010101u;
        v.w = (((bits >> 12) & 0xFu) * 0x00204081u) & 0x01010101u;
        reinterpret_cast<uint4*>(out)[q] = v;
      }
    } else {
      for (int d = C.sub; d < DPE; d += NT) {
        const int i = 4 * d, jb = i / EE, o = i - jb * EE;
        const uint64_t w = (uint64_t)cl[jb] | ((uint64_t)(jb + 1 < NB ? cl[jb + 1] : 0u) << EE);
        out[d] = ((uint32_t)(w >> o) & 0xFu) * 0x00204081u & 0x01010101u;
      }
    }
    return;
  }
  // ---- dwords of the wave's obs run
  constexpr int DPE = NB * EE / 4;       // dwords per env (a cell is one byte)
  constexpr int D = EPW * DPE;           // dwords per wave
  const int e_first = blockIdx.x * EPW;  // the wave's first env
  uint32_t* out = reinterpret_cast<uint32_t*>(obs_out + (size_t)e_first * (NB * EE));
  const int lane = (int)(threadIdx.x & 63);
  // three dwords per lane when an env's run is whole triples and the wave's
  // triples fit 64 lanes (C2: 25 per env): one pair of ds_bpermutes and one
  // global_store_dwordx3 per lane; a triple's 12 bits span at most two crops
  constexpr int TPE = DPE / 3;  // dword triples per env
  constexpr bool X3 = DPE % 3 == 0 && EPW * TPE <= 64 && EE >= 12;
  if constexpr (X3) {
    const int es = EPW == 1 ? 0 : lane / TPE;  // env slot of the lane's triple
    const int b0 = 12 * (lane - es * TPE);     // its first bit within that env's stream
    const int jb = b0 / EE, o = b0 - jb * EE;
    const int src = es * LPE + jb;
    const uint32_t w0 = (uint32_t)__shfl((int)crop, src);
    const uint32_t w1 = (uint32_t)__shfl((int)crop, src + 1 < 64 ? src + 1 : src);
    const uint32_t bits = (uint32_t)((((uint64_t)w1 << EE) | w0) >> o);
    if (lane < EPW * TPE && e_first + es < s.B) {
      typedef uint32_t u32x3 __attribute__((ext_vector_type(3), aligned(4)));
      u32x3 v;
      v.x = ((bits & 0xFu) * 0x00204081u) & 0x01010101u;
      v.y = (((bits >> 4) & 0xFu) * 0x00204081u) & 0x01010101u;
      v.z = (((bits >> 8) & 0xFu) * 0x00204081u) & 0x01010101u;
      *reinterpret_cast<u32x3*>(out + 3 * lane) = v;
    }
  } else {
#pragma unroll
    for (int d0 = 0; d0 < D; d0 += 64) {
      const int d = d0 + lane;
      const int es = EPW == 1 ? 0 : d / DPE;  // env slot of dword d
      const int i = 4 * (d - es * DPE);       // its first bit within that env's stream
      const int jb = i / EE, o = i - jb * EE;
      const int src = es * LPE + jb;
      const uint32_t w0 = (uint32_t)__shfl((int)crop, src);
      const uint32_t w1 = (uint32_t)__shfl((int)crop, src + 1 < 64 ? src + 1 : src);
      const uint32_t nib = ((w0 | (w1 << EE)) >> o) & 0xFu;
      if (d < D && e_first + es < s.B) out[d] = (nib * 0x00204081u) & 0x01010101u;
    }
  }
}

// --------------------------------------------------------------------------
// the env kernel: EPW envs per workgroup
// --------------------------------------------------------------------------
// minimum waves per SIMD the compiler must leave room for (VGPR budget):
// one env per 4-wave workgroup at C4, LDS-bound at 5 workgroups per CU
template <int NT, class SH>
constexpr int env_min_waves() {
#ifdef MC_C4_WPE
  if (NT == 256 && SH::NB == 360) return MC_C4_WPE;
#endif
  // C5 (16 agents): the robots in registers for the moves and the obs crops
  // would take the kernel past 128 VGPRs (3 waves per SIMD); keep 4
// (round 5, profiles/r5/wpe/: 5 waves per SIMD spill 10 VGPRs, 82.1 ->
// 87.3 us at the C5 steady state; 6 spill 28, 117.9 us)
#ifdef MC_C5_WPE  // A/B knob: waves per SIMD the C5 shape must fit
  if (SH::N == 16) return MC_C5_WPE;
#endif
  return SH::N == 16 ? 4 : 1;
}

template <int NT, int EPW, typename WT, class SH>
__global__ __launch_bounds__(NT, (env_min_waves<NT, SH>())) void env_kernel(EnvArgs args) {
  State s = args.s;
  specialize<SH>(s);
  EnvIO io = args.io;
  const int mode = io.mode;
  using CtxT = Ctx<NT, EPW, WT>;
  constexpr int LPE = CtxT::LPE;
  constexpr int KI = CtxT::KI;
  // march steps per batch: the whole march when the shape fixes a short
  // beam_kmax, a quarter of a long one (register pressure)
  constexpr int SUK0 = (SH::KM > 0 && SH::KM <= 12) ? SH::KM : (SH::KM > 12 ? (SH::KM + 3) / 4 : 8);
  constexpr int NSM = (SH::N > 0 && SH::N <= 8) ? SH::N : 0;  // compile-time agent count, if small
  // rays per lane per march pass: 3 where that saves a pass over the
  // default (C5: 336 rays over 128 lanes, one pass of 3 instead of two of 2)
  constexpr int RPLK = MC_RPL_SHAPE && SH::N > 0 && SH::NB > 0 && SH::NB < 64 && EPW == 1 &&
                               (SH::N * SH::NB + 3 * NT - 1) / (3 * NT) < (SH::N * SH::NB + CtxT::RPL * NT - 1) / (CtxT::RPL * NT)
                           ? 3
                           : 0;
  // (3 rays per lane: half the march's batch, the row words of a batch stay
  // within the register budget)
  constexpr int SUK = RPLK == 3 ? (SUK0 + 1) / 2 : SUK0;
  // compiled shapes with up to 8 agents: map byte offsets fit 32 bits
  // (launch_env checks; the C5 shape's maps pass 4 GB)
  constexpr bool O32 = SH::N > 0 && SH::N <= 8;
  // register front (front_regs / moves_front): compiled agent count <= 8,
  // one wave per workgroup
  constexpr bool FRONT = NSM > 0 && NT == 64;
  // moves from registers in the first wave of a multi-wave env during round
  // trip 2 (compiled agent count <= 8, lidar: C4)
  constexpr bool EARLY = NSM > 0 && NT > 64 && EPW == 1 && SH::NB > 0;
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
      state_lds_bytes(s, (int)sizeof(WT));
  C.L = carve<WT>(smem + slot * slot_stride(slot_lds), s);
  const Lds<WT>& L = C.L;
  const int e = C.e;

  const bool is_step = mode == MODE_STEP;

  STAMP(0);
  // ---- round trip 1: positions, actions, scalars, beam table.  Every load
  // is issued (unpredicated, clamped addresses) before any result is used:
  // one round trip, not one per branch.
  // (register front with QUAD: every lane loads robot sub % N, so each quad
  // holds all robots; other lanes of other builds read robot 0)
  const int ag = (FRONT && FrontQuad<NSM>::ok) ? (C.sub & (N - 1)) : (C.sub < N ? C.sub : 0);
  // absent inputs read a harmless valid byte instead (no branch, no wait)
  const uint8_t* ab = is_step ? io.actions : reinterpret_cast<const uint8_t*>(s.pos);
  const uint32_t eN = (uint32_t)e * (uint32_t)N;
  const uint8_t* mb = io.env_mask != nullptr ? io.env_mask + e : reinterpret_cast<const uint8_t*>(s.pos);
  const int2 p0 = el<O32>(reinterpret_cast<const int2*>(s.pos), eN + ag);
  const int act_raw = el<O32>(ab, is_step ? eN + ag : 0), act0_raw = el<O32>(ab, is_step ? eN : 0);
  const int req_raw = mb[0];
  const int g0 = el<O32>(s.env_grid, e);
  const uint64_t moved0 = el<O32>(s.moved, e);
  const uint32_t free_old = el<O32>(s.free_cnt, e), vis_old = el<O32>(s.vis_cnt, e);
  const int currstep0 = el<O32>(s.currstep, e);
  const double dthresh0 = el<O32>(s.done_thresh, e);
  const bool lidar = s.sensor == 0;
  const int nbl = lidar ? s.nbeams : 1;  // a square env reads a dummy record
  const int4 bm0 = reinterpret_cast<const int4*>(lidar ? (const void*)s.beams : (const void*)s.pos)
      [C.sub < nbl ? C.sub : 0];
  // fan march: the fan data (LUTs, sector and special records) instead of the
  // beam records, up to 3 * LPE int4 in this round trip
  const bool fan = fan_on(s);
  const int n16 = fan ? s.fan_words / 4 : 0;
  const int4* fsrc = reinterpret_cast<const int4*>(fan ? (const void*)s.fan_data : (const void*)s.pos);
  const int4 fv0 = fsrc[C.sub < n16 ? C.sub : 0];
  const int4 fv1 = fsrc[C.sub + LPE < n16 ? C.sub + LPE : 0];
  const int4 fv2 = fsrc[C.sub + 2 * LPE < n16 ? C.sub + 2 * LPE : 0];
  // dist_reward: M and witness of each free map, and the top-cell cache's
  // count and box (mc_internal.h State::dist_ch), in the same round trip
  const int agd = C.sub < N ? C.sub : 0;
  int2 mwv = make_int2(-1, 0);
  int4 chd = make_int4(-1, 0, 0, 0);
  int2 chb = make_int2(0, 0);
  if (s.dist) mwv = reinterpret_cast<const int2*>(s.dist_mw)[eN + agd];
  if (s.dist_ch) {
    const int4* hp = reinterpret_cast<const int4*>(s.dist_ch + ((size_t)eN + agd) * 8);
    chd = hp[0];
    chb = *reinterpret_cast<const int2*>(hp + 1);
  }
  zero_marks<NT, EPW, WT>(s, C);  // overlaps the round trip
  // every result is needed below: keep the compiler from sinking a load into
  // the branch that uses it (that would make it a round trip of its own)
  asm volatile("" ::"v"(p0.x), "v"(p0.y), "v"(act_raw), "v"(act0_raw), "v"(req_raw), "v"(g0),
               "v"(bm0.x), "v"(bm0.w), "v"(mwv.x), "v"(mwv.y), "v"(chd.x), "v"(chd.w), "v"(chb.y));
  const int act = is_step ? act_raw : 255;
  // one env per workgroup: the env's flags are uniform -- made scalar
  // (readfirstlane), their branches are scalar branches instead of lane masks
  // kept in SGPR pairs (MC_UNIFORM_FLAGS)
  auto uni = [](int v) { return (EPW == 1 && MC_UNIFORM_FLAGS) ? __builtin_amdgcn_readfirstlane(v) : v; };
  const int act0 = uni(is_step ? act0_raw : 0);  // agent 0's byte: the sentinel
  const int req = uni(io.env_mask != nullptr ? req_raw : 1);

  const bool sentinel = valid && is_step && act0 == 255;
  const bool reset_req = valid && !is_step && req != 0;
  const bool active = valid && is_step && !sentinel;
  const bool sent_reset = sentinel && s.auto_reset;  // a sentinel's done resets too
  // dist_reward: this lane's agent (C.sub < N) goes to the full transform's list
  bool dlist = false;
  if (C.sub < N) {
    set_agent<WT>(s, L, C.sub, p0.x, p0.y);
    L.act[C.sub] = (uint8_t)act;
  }
  if (C.sub == 0) {
    L.sc->grid = g0;
    L.sc->moved = moved0;
    L.sc->pen = 0.0;
    L.sc->cnt_free = 0;
    L.sc->cnt_vis = 0;
    L.sc->do_reset = 0;
    L.sc->dist_hit = 0;
    L.sc->dist_fail = 0;
    L.sc->zero = 0;
    if constexpr (EPW == 1 && MC_UNIFORM_FLAGS)
      L.sc->path = (active ? kPathActive : 0) | (reset_req ? kPathResetReq : 0) | (sent_reset ? kPathSentReset : 0) |
                   (sentinel ? kPathSentinel : 0);
  }
  if (s.dist && C.sub < N) {  // dist_reward: M and witness of each free map
    L.dm[C.sub] = mwv.x;
    L.dw[C.sub] = mwv.y;
  }
  // (chd / chb: the top-cell cache of agent C.sub; its box grows by this
  // step's sensing window below)
  if (fan) {
    int4* dst = reinterpret_cast<int4*>(L.fan);
    if (C.sub < n16) dst[C.sub] = fv0;
    if (C.sub + LPE < n16) dst[C.sub + LPE] = fv1;
    if (C.sub + 2 * LPE < n16) dst[C.sub + 2 * LPE] = fv2;
    for (int j = C.sub + 3 * LPE; j < n16; j += LPE) dst[j] = fsrc[j];
  } else if (lidar) {
    if (C.sub < s.nbeams) reinterpret_cast<int4*>(L.beams)[C.sub] = bm0;
    for (int b = C.sub + LPE; b < s.nbeams; b += LPE) L.beams[b] = s.beams[b];
  }
  __syncthreads();
  reload_state<SH, EPW>(s, io);

  if (active) {
    STAMP(1);
    Items<KI> I;
    if constexpr (FRONT) {
      // ---- round trip 2, issue: the robots' target-cell grid tiles first
      // (the moves wait only for them), then every staged tile; block
      // origins and moves from registers (front_regs)
      Front<NSM> F;
      front_regs<NT, EPW, WT, NSM>(s, C, p0.x, p0.y, act, F);
      const int dx = (act == 0) - (act == 2), dy = (act == 1) - (act == 3);
      const int tx = p0.x + dx, ty = p0.y + dy;
      const bool inb = (unsigned)tx < (unsigned)s.Wp && (unsigned)ty < (unsigned)s.Lp;
      const uint64_t tt = ld_tile<O32>(s.grid_neg, __umul24((uint32_t)g0, (uint32_t)s.MT) +
                                                       tile_index24(s.TCS, inb ? tx >> 3 : 0, inb ? ty >> 3 : 0));
      stage_load<NT, EPW, WT, KI, O32, NSM>(s, C, g0, true, I, &F);
      moves_front<NT, EPW, WT, NSM>(s, C, F, !inb || ((tt >> tile_bit(tx, ty)) & 1ull),
                                    (uint32_t)tx | ((uint32_t)ty << 16), act, moved0, -s.pen);
      stage_scatter<NT, EPW, WT, KI>(s, C, I);
    } else if constexpr (EARLY) {
      // ---- round trip 2 with the moves of a multi-wave env: the first wave
      // moves the robots from registers (front_regs / moves_front: lane i
      // holds robot i, its target-cell grid tile loaded first) while the
      // staged tiles are in flight; the other waves only stage
      const int dx = (act == 0) - (act == 2), dy = (act == 1) - (act == 3);
      const int tx = p0.x + dx, ty = p0.y + dy;
      const bool inb = (unsigned)tx < (unsigned)s.Wp && (unsigned)ty < (unsigned)s.Lp;
      const uint64_t tt = ld_tile<O32>(s.grid_neg, __umul24((uint32_t)g0, (uint32_t)s.MT) +
                                                       tile_index24(s.TCS, inb ? tx >> 3 : 0, inb ? ty >> 3 : 0));
      stage_load<NT, EPW, WT, KI, O32>(s, C, g0, true, I);
      STAMP(15);  // loads issued (the first wave's moves follow)
      if (C.sub < 64) {
        Front<NSM> F;
        front_regs<NT, EPW, WT, NSM>(s, C, p0.x, p0.y, act, F);
        moves_front<NT, EPW, WT, NSM>(s, C, F, !inb || ((tt >> tile_bit(tx, ty)) & 1ull),
                                      (uint32_t)tx | ((uint32_t)ty << 16), act, moved0, -s.pen);
      }
      stage_scatter<NT, EPW, WT, KI>(s, C, I);
    } else {
      stage<NT, EPW, WT, KI, O32>(s, C, g0, true, I);  // ---- round trip 2 ----
    }
    // count_nonzero(grid > 0) for percent_covered: kept in a register until
    // the reward (no wait here)
    const int numfree = el<O32>(s.numfree, g0);
    __syncthreads();
    STAMP(2);
    reload_state<SH, EPW>(s, io);
    // (the same loop on the scalar unit, robots read by v_readlane, was
    // slower: 10.17 vs 9.83 us at C2 -- +178 SALU for -17 VALU per wave)
    if constexpr (!FRONT && !EARLY) {  // (FRONT, EARLY: moved during round trip 2)
      // the first wave of the slot moves the robots (lane 0 publishes); the
      // other waves of a multi-wave workgroup only wait at the barrier
      // (C5, 16 agents: moves_regs took 17.7k vs 7.3k cycles per wave -- the
      // every-lane replay of 256 position compares outweighs the broadcasts;
      // the loop on the scalar unit from v_readlane copies, 111.3 vs 107.8 us
      // per env kernel, profiles/r4/c5_grid/)
      if constexpr (SH::N > 0 && SH::N <= 8) {
        if (NT == 64 || C.sub < 64) moves_regs<NT, EPW, WT, SH::N>(s, C, -s.pen);
      } else if constexpr (SH::N > 8 && EPW == 1 && !MC_MOVES_SERIAL) {
        if (C.sub < 64) moves_par<NT, EPW, WT, SH::N>(s, C, -s.pen);
      } else if (C.sub < 64) {
        moves<NT, EPW, WT>(s, C, -s.pen);
      }
      __syncthreads();
    }
    STAMP(3);
    reload_state<SH, EPW>(s, io);
    // dist_reward: lane i < N loads its agent's PRE terms (the last step's
    // dist kernels wrote them) now that its move is known; they land during
    // the sensing
    // (compiled shapes; the generic kernels keep the loads in the reward:
    // two more live registers there cost the u64 ones a wave per SIMD)
    constexpr bool kPrePrefetch = SH::N > 0;
    // one env per workgroup: the env's counters re-read here (they land
    // during the sensing) rather than kept from round trip 1 in SGPRs,
    // which spilled (nothing writes them before the reward)
    uint32_t free_old_r = free_old, vis_old_r = vis_old;
    int currstep_r = currstep0;
    double dthresh_r = dthresh0;
    if constexpr (EPW == 1 && MC_UNIFORM_FLAGS) {
      free_old_r = el<O32>(s.free_cnt, e);
      vis_old_r = el<O32>(s.vis_cnt, e);
      currstep_r = el<O32>(s.currstep, e);
      dthresh_r = el<O32>(s.done_thresh, e);
    }
    float dpre0 = 0.0f, dprek = 0.0f;
    if (kPrePrefetch && s.dist && C.sub < N) {
      const int dx = L.x[C.sub] - L.x0[C.sub], dy = L.y[C.sub] - L.y0[C.sub];
      const int k = dx == 1 ? 1 : (dy == 1 ? 2 : (dx == -1 ? 3 : (dy == -1 ? 4 : 0)));
      const float* pr = s.dist_pre + ((size_t)e * N + C.sub) * 8;
      dpre0 = pr[0];
      dprek = pr[1 + k];
    }
    sense_and_merge<NT, EPW, WT, KI, SUK, NSM, SH::KN, SH::KM, RPLK>(s, C, I, Reload<SH, EPW>());
    __syncthreads();
    STAMP(5);
    reload_state<SH, EPW>(s, io);
    // every lane of the slot computes the reward and done (the same values:
    // no broadcast round trip or barrier before the stores); lane 0 stores
    bool do_reset;
    {
      Scal* c = L.sc;
      const uint32_t fc = free_old_r + c->cnt_free;
      const uint32_t vc = vis_old_r + c->cnt_vis;
      const int cs = currstep_r + 1;                         // :154
      // observe() :206-258 returns the float32 sum of the agents' distance
      // terms (dist_reward, agent order) plus the union delta (float64)
      // (only lane 0's value is stored: the agents' terms are in the slot's
      // first lanes, N <= 64, and are summed in agent order)
      float dsum = 0.0f;
      if (s.dist) {
        if constexpr (kPrePrefetch) {
          const float term = dist_value(dprek, dpre0);  // :222-223,239-240
          for (int i = 0; i < N; ++i)
            dsum = __fadd_rn(dsum, __builtin_bit_cast(float, bcast(C, __builtin_bit_cast(int, term), i)));
        } else {
          for (int i = 0; i < N; ++i) {
            const int dx = L.x[i] - L.x0[i], dy = L.y[i] - L.y0[i];
            const int k = dx == 1 ? 1 : (dy == 1 ? 2 : (dx == -1 ? 3 : (dy == -1 ? 4 : 0)));
            const float* pr = s.dist_pre + ((size_t)e * N + i) * 8;
            dsum = __fadd_rn(dsum, dist_value(pr[1 + k], pr[0]));  // :222-223,239-240
          }
        }
      }
      const double obs_reward = (double)dsum + (double)c->cnt_vis;
      double r = c->pen + obs_reward;                        // :120,132-151
      double dt = dthresh_r;
      const double thr = (1.0 < dt) ? 1.0 : dt;              // min(done_thresh, 1)
      // pc = count/numfree (:552), correctly rounded; thr <= pc.  With thr
      // == 1 (the default) the test is fc >= numfree exactly (counts are
      // < 2^24: a quotient below 1 rounds below 1), so the float64 divide
      // runs only when the threshold or the episode record needs it.  A
      // grid with no cell > 0 takes the division: 0/0 = NaN is never covered,
      // as in the reference
      const bool exact1 = thr == 1.0 && numfree > 0;
      double pc = 0.0;
      if (!exact1) pc = (double)fc / (double)numfree;
      const bool covered = exact1 ? fc >= (uint32_t)numfree : thr <= pc;
      if (covered) r += s.term;                              // :156-157
      bool done = false;
      if (covered) { dt += s.dincr; done = true; }           // :540-543
      else if (cs == s.maxsteps) done = true;                // :544-545
      do_reset = uni((int)(done && s.auto_reset)) != 0;
      if (C.sub == 0) {
        el<O32>(io.reward_out, e) = r;
        el<O32>(io.done_out, e) = done ? 1 : 0;
        if (done) {  // the episode record (Utils/utils.py:138-141)
          el<O32>(s.ep_pc, e) = exact1 ? (double)fc / (double)numfree : pc;
          el<O32>(s.ep_len, e) = cs;
        }
        el<O32>(s.free_cnt, e) = fc;
        el<O32>(s.vis_cnt, e) = vc;
        el<O32>(s.currstep, e) = cs;
        el<O32>(s.done_thresh, e) = dt;
        c->do_reset = do_reset ? 1 : 0;
      }
    }
    // dist_reward: the POST terms of the maps whose M is still known (the
    // others, and a reset env's, go to the full transform's list)
    if (s.dist) {
      const uint64_t skip = do_reset ? ~0ull : L.sc->dist_hit;  // (and every agent with M < 0)
      // dist_window overwrites dist_pre with the POST terms; without the
      // prefetch every lane of the slot read all agents' PRE terms in the
      // reward above, and in a multi-wave slot another wave may still be
      // there: every wave passes the reward before any POST store
      if constexpr (NT > 64 && !kPrePrefetch) __syncthreads();
      if (MC_ABL != 1) {
        // (tried, round 5: one lane per (agent, target row) growing the
        // row's covered set by a bit-parallel dilation -- 83.6 against 81.7
        // us at the C5 steady state, profiles/r5/win/; removed)
        if constexpr (Ctx<NT, EPW, WT>::LPE % 32 == 0 && MC_DIST_AM) {
          if constexpr (MC_DIST_AM2 && SH::N > 0 && SH::N <= 64) {
            if (5 + s.E * s.E <= 32) dist_window_am2<NT, EPW, WT, SH::N>(s, C, skip);
            else dist_window<NT, EPW, WT>(s, C, skip);
          } else {
            if (5 + s.E * s.E <= 32) dist_window_am<NT, EPW, WT>(s, C, skip);
            else dist_window<NT, EPW, WT>(s, C, skip);
          }
        } else {
          dist_window<NT, EPW, WT>(s, C, skip);
        }
      }
      __syncthreads();
      dlist = C.sub < N && ((((skip | L.sc->dist_fail) >> C.sub) & 1ull) || L.dm[C.sub] < 0);
    }
    // several waves: the slot's Scal reads above come before reset_env's
    // writes (one wave: its LDS operations complete in order)
    if constexpr (NT > 64) __syncthreads();
    STAMP(6);
    reload_state<SH, EPW>(s, io);
    if (!do_reset) {
      store_tiles<NT, EPW, WT, KI, O32>(s, C, I);
      STAMP(7);
    } else {
      reset_env<NT, EPW, WT, SUK, NSM, SH::KN, O32, SH::KM, RPLK>(s, C, nullptr, Reload<SH, EPW>());  // the finished episode's tiles are not stored
    }
  } else if (reset_req || sent_reset) {
    reload_state<SH, EPW>(s, io);
    if (C.sub == 0 && sentinel) {  // the sentinel's done ends the episode (utils.py:22,41)
      io.reward_out[e] = 0.0;
      io.done_out[e] = 1;
      s.ep_pc[e] = (double)free_old / (double)s.numfree[g0];
      s.ep_len[e] = currstep0;
    }
    reset_env<NT, EPW, WT, SUK, NSM, SH::KN, O32, SH::KM, RPLK>(s, C, reset_req ? io.inj_pos : nullptr, Reload<SH, EPW>());
    dlist = s.dist && C.sub < N;  // fresh maps: M unknown
  } else {
    // sentinel step without auto-reset / env left out of a partial reset:
    // obs of the current state only (dec_grid_rl.py:104-107,160).  Only the
    // old free / obstacle tiles are needed (fold / oold): no row or column
    // plane is scattered.  With the fan march the column planes overlay
    // fold / oold (carve), and a multi-wave slot's column-byte stores would
    // race with another wave's stage_fold stores.
    reload_state<SH, EPW>(s, io);
    Items<KI> I;
    stage_load<NT, EPW, WT, KI, O32>(s, C, g0, true, I);
    stage_fold<NT, EPW, WT, KI>(s, C, I);
    // unchanged maps keep their dist terms; an unknown M (a state upload)
    // needs the full transform
    dlist = s.dist && C.sub < N && L.dm[C.sub] < 0;
    if (C.sub == 0 && sentinel) {
      io.reward_out[e] = 0.0;
      io.done_out[e] = 1;
      s.ep_pc[e] = (double)free_old / (double)s.numfree[g0];
      s.ep_len[e] = currstep0;
    }
  }
  __syncthreads();

  // the branch flags again, from LDS: one env per workgroup keeps them out of
  // SGPR pairs across the branch (MC_UNIFORM_FLAGS)
  const int path = L.sc->path;
  constexpr bool kPathLds = EPW == 1 && MC_UNIFORM_FLAGS;
  const bool p_active = kPathLds ? (path & kPathActive) != 0 : active;
  const bool p_reset_req = kPathLds ? (path & kPathResetReq) != 0 : reset_req;
  const bool p_sent_reset = kPathLds ? (path & kPathSentReset) != 0 : sent_reset;
  if (p_active || p_reset_req || p_sent_reset) {
    if (C.sub < N)
      el<O32>(reinterpret_cast<int2*>(s.pos), (uint32_t)e * (uint32_t)N + C.sub) = make_int2(L.x[C.sub], L.y[C.sub]);
    if (C.sub == 0) el<O32>(s.moved, e) = L.sc->moved;
    // dist_reward: a reset map, or one whose witness got closer than M,
    // has an unknown M now (recomputed by the full transform, mc_dist.hip)
    if (s.dist && C.sub < N &&
        (p_reset_req || p_sent_reset || L.sc->do_reset || ((L.sc->dist_hit >> C.sub) & 1ull)))
      s.dist_mw[((size_t)e * N + C.sub) * 2] = -1;
    if (s.dist_ch && C.sub < N) {
      int* hp = s.dist_ch + ((size_t)e * N + C.sub) * 8;
      if (p_reset_req || p_sent_reset || L.sc->do_reset) {
        hp[0] = -1;  // the map was cleared: the cached cells' d are stale
      } else if (chd.x > 0) {  // every newly covered cell lies in the sensing window
        const int x = L.x[C.sub], y = L.y[C.sub], H = s.H;
        *reinterpret_cast<int4*>(hp) = make_int4(chd.x, chd.y, min(chd.z, x - H), min(chd.w, y - H));
        *reinterpret_cast<int2*>(hp + 4) = make_int2(max(chb.x, x + H), max(chb.y, y + H));
      }
    }
  }
  if (s.dist) {
    // the full transform's work list (mc_dist.hip launch_dist_listed): one
    // atomic per env slot of the wave on its env's shard (e % kListShards,
    // spread over kListShards lines: early after a reset nearly every env
    // appends, ~8k returning atomics per step on one address), the slot's
    // entries at consecutive places of the shard
    const bool me = valid && dlist;
    const uint64_t m = __ballot(me);
    if (m) {
      const int lane = (int)(threadIdx.x & 63);
      const uint64_t slotm = LPE >= 64 ? ~0ull : (low_mask(LPE) << (lane & ~(LPE - 1) & 63));
      const uint64_t ms = m & slotm;
      if (ms) {
        const int leader = __ffsll((unsigned long long)ms) - 1;
        const uint32_t sh = (uint32_t)e % (uint32_t)kListShards;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(s.dist_shc + sh * kShardStride, (uint32_t)__popcll(ms));
        base = (uint32_t)__shfl((int)base, leader);
        if (me)
          s.dist_cnt[5 + sh * s.dist_cap + base + __popcll(ms & ((1ull << lane) - 1ull))] =
              (uint32_t)e * (uint32_t)N + (uint32_t)C.sub;
      }
    }
    if (s.dist_full && blockIdx.x == 0 && threadIdx.x == 0) {  // the last step's full list is done
      s.dist_full[2] = s.dist_full[0];
      s.dist_full[0] = 0;
    }
  }
  STAMP(8);
  reload_state<SH, EPW>(s, io);
  if constexpr (ObsFast<SH::EGO, SH::N, SH::LC>::ok && (NT == 64 || EPW == 1) &&
                ObsFast<SH::EGO, SH::N, SH::LC>::NB <= 64) {
    if (MC_ABL != 4) write_obs_fast<NT, EPW, WT, SH::N, SH::EGO, SH::LC>(s, C, io.obs_out);  // every lane of the workgroup
  } else {
    if (valid) write_obs<NT, EPW, WT, (SH::N > 0 && SH::N <= 16) ? SH::N : 0>(s, C, io.obs_out);
  }
  STAMP(9);
  if (valid && io.adj_out != nullptr) {  // updateCommmunicationGraph (:374-391)
    uint8_t* ad = io.adj_out + (size_t)e * N * N;
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

// Envs per wave: two when an env fits 32 lanes (N <= 32, at most KI staged
// tiles and 3 beams per lane), else one env per workgroup of NT threads.
int env_pack(const State& s) {
  const int items = s.N * s.TW * s.TW;
  const int rays = s.sensor == 0 ? s.N * s.nbeams : 0;
  return (s.N <= 32 && items <= kMaxItemsPerLane * 32 && rays <= 3 * 32) ? 2 : 1;
}


// MARLCOV_SPECIALIZE=0 forces the generic (runtime-shape) kernels (A/B tests)
static bool getenv_spec() {
  static const bool on = [] {
    const char* v = getenv("MARLCOV_SPECIALIZE");
    return !(v && v[0] == '0');
  }();
  return on;
}

// One env-kernel instantiation: its name (mc_kernel_variant) and launcher.
struct EnvLaunch {
  const char* name;
  void (*launch)(const State& s, int mode, const uint8_t* actions, const uint8_t* env_mask,
                 const int32_t* inj_pos, double* reward, uint8_t* done, uint8_t* obs, uint8_t* adj,
                 hipStream_t stream);
};

template <int T, int P, typename W, class SH>
static void launch_one(const State& s, int mode, const uint8_t* actions, const uint8_t* env_mask,
                       const int32_t* inj_pos, double* reward, uint8_t* done, uint8_t* obs, uint8_t* adj,
                       hipStream_t stream) {
  const size_t slot_lds = state_lds_bytes(s, (int)sizeof(W));
  const EnvArgs args{s, EnvIO{actions, env_mask, inj_pos, reward, done, obs, adj, mode}};
  hipLaunchKernelGGL((env_kernel<T, P, W, SH>), dim3((s.B + P - 1) / P), dim3(T), slot_stride(slot_lds) * P,
                     stream, args);
}

using Dynamic = Shape<0, 0, 0, 0, 0>;
using ShapeC2 = Shape<4, 10, 21, 2, 10, 8>;      // the bench workload
using ShapeC2D = Shape<4, 10, 21, 2, 10, 8, 4>;  // C2 + dijkstra_input (4 obs layers)
// 360 beams, R=20; its fan: 64 sector slots, 2 special
// beams, 1,024 LUT words + 32 pair records x 42 + 2 x 8 = 2,384 words
using ShapeC4 = Shape<8, 20, 360, 2, 20, 15, 3, 0, 64, 2, 2384>;
using ShapeC4R = Shape<8, 20, 360, 2, 20, 15>;  // the same without a baked fan (the ray march: MARLCOV_FAN=0)
// the bench instantiations (bench.py CONFIGS: 256x256 / 128x128 / 512x512
// grids, auto-reset, no comm graph); other grids run the shapes above
using ShapeC4B = Shape<8, 20, 360, 2, 20, 15, 3, 0, 64, 2, 2384, 258>;
using ShapeC2B = Shape<4, 10, 21, 2, 10, 8, 3, 0, 0, 0, 0, 130>;
using ShapeC5B = Shape<16, 10, 21, 2, 10, 8, 4, 1, 0, 0, 0, 514>;
using ShapeC5 = Shape<16, 10, 21, 2, 10, 8, 4, 1>;  // 16 agents, egoradius 2, dist_reward (4 obs layers)

#ifndef MC_BENCH_SHAPES  // build knob (A/B): 0 leaves the grid-baked bench instantiations out
#define MC_BENCH_SHAPES 1
#endif
constexpr bool kBenchShapes = MC_BENCH_SHAPES != 0;

#define MC_EL(T, P, W, SH, NAME) \
  EnvLaunch { "env_kernel<" #T "," #P "," NAME ">", &launch_one<T, P, W, SH> }

// The instantiation for this state: compiled shapes when the runtime State
// matches one exactly (and its map offsets fit 32 bits), else the generic
// kernel for the lane count / envs per workgroup.
EnvLaunch select_env(const State& s, int nt, int epw) {
  const bool narrow = s.TW <= 4;  // window rows fit a u32
  // compiled shapes address the map arrays with 32-bit byte offsets
  const uint64_t mtb = (uint64_t)s.MT * 8;
  const bool fits32 = (uint64_t)s.B * s.N * mtb < (1ull << 32) && (uint64_t)s.G * mtb < (1ull << 32);
  const bool spec = getenv_spec();
  if (epw == 2) {
    if (narrow && fits32 && spec && kBenchShapes && ShapeC2B::matches(s)) return MC_EL(64, 2, uint32_t, ShapeC2B, "u32,C2");
    if (narrow && fits32 && spec && ShapeC2::matches(s)) return MC_EL(64, 2, uint32_t, ShapeC2, "u32,C2");
    if (narrow && fits32 && spec && ShapeC2D::matches(s)) return MC_EL(64, 2, uint32_t, ShapeC2D, "u32,C2D");
    if (narrow) return MC_EL(64, 2, uint32_t, Dynamic, "u32,generic");
    return MC_EL(64, 2, uint64_t, Dynamic, "u64,generic");
  }
  if (narrow) {
    if (nt == 64 && fits32 && spec && ShapeC2::matches(s)) return MC_EL(64, 1, uint32_t, ShapeC2, "u32,C2");
    if (nt == 64 && fits32 && spec && ShapeC2D::matches(s)) return MC_EL(64, 1, uint32_t, ShapeC2D, "u32,C2D");
    if (nt == 128 && spec && kBenchShapes && ShapeC5B::matches(s)) return MC_EL(128, 1, uint32_t, ShapeC5B, "u32,C5");
    if (nt == 128 && spec && ShapeC5::matches(s)) return MC_EL(128, 1, uint32_t, ShapeC5, "u32,C5");
    switch (nt) {
      case 64: return MC_EL(64, 1, uint32_t, Dynamic, "u32,generic");
      case 128: return MC_EL(128, 1, uint32_t, Dynamic, "u32,generic");
      case 256: return MC_EL(256, 1, uint32_t, Dynamic, "u32,generic");
      case 512: return MC_EL(512, 1, uint32_t, Dynamic, "u32,generic");
      default: return MC_EL(1024, 1, uint32_t, Dynamic, "u32,generic");
    }
  }
  if (nt == 256 && fits32 && spec && kBenchShapes && ShapeC4B::matches(s)) return MC_EL(256, 1, uint64_t, ShapeC4B, "u64,C4");
  if (nt == 256 && fits32 && spec && ShapeC4::matches(s)) return MC_EL(256, 1, uint64_t, ShapeC4, "u64,C4");
  if (nt == 256 && fits32 && spec && ShapeC4R::matches(s)) return MC_EL(256, 1, uint64_t, ShapeC4R, "u64,C4");
  switch (nt) {
    case 64: return MC_EL(64, 1, uint64_t, Dynamic, "u64,generic");
    case 128: return MC_EL(128, 1, uint64_t, Dynamic, "u64,generic");
    case 256: return MC_EL(256, 1, uint64_t, Dynamic, "u64,generic");
    case 512: return MC_EL(512, 1, uint64_t, Dynamic, "u64,generic");
    default: return MC_EL(1024, 1, uint64_t, Dynamic, "u64,generic");
  }
}
#undef MC_EL

const char* env_variant(const State& s, int nt, int epw) { return select_env(s, nt, epw).name; }

hipError_t launch_env(const State& s, int mode, const uint8_t* actions, const uint8_t* env_mask,
                      const int32_t* inj_pos, double* reward, uint8_t* done, uint8_t* obs,
                      uint8_t* adj, int nt, int epw, hipStream_t stream) {
  select_env(s, nt, epw).launch(s, mode, actions, env_mask, inj_pos, reward, done, obs, adj, stream);
  return hipGetLastError();
}

}  // namespace mc
