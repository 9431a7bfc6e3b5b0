// mc_capi.hip — the extern "C" boundary of libmarlcov.so (include/marlcov.h).
// Owns the device state of a batch of envs and launches mc_kernels.hip.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <algorithm>
#include <vector>

#include "marlcov.h"
#include "mc_internal.h"

namespace mc {
hipError_t launch_env(const State& s, int mode, const uint8_t* actions, const uint8_t* env_mask,
                      const int32_t* inj_pos, double* reward, uint8_t* done, uint8_t* obs,
                      uint8_t* adj, int nt, int epw, hipStream_t stream);
int env_pack(const State& s);
hipError_t launch_share(const State& s, const uint8_t* actions, hipStream_t stream);
hipError_t launch_pack(const State& s, const int8_t* grids, hipStream_t stream);
hipError_t launch_gen(const State& s, uint64_t seed, double p, hipStream_t stream);
hipError_t launch_random_actions(const State& s, uint64_t seed, int step, uint8_t* out, hipStream_t stream);
const char* env_variant(const State& s, int nt, int epw);
hipError_t launch_dijkstra(const State& s, int pad, int layer, int Lc, uint8_t* obs,
                           uint32_t* list, bool window, hipStream_t stream);
hipError_t launch_dist(const State& s, int pad, int post, float* pre_out, float* dist_obs,
                       hipStream_t stream);
hipError_t launch_dist_listed(const State& s, int pad, float* pre_out, float* dist_obs,
                              uint32_t* list, uint32_t* count, uint32_t* full, hipStream_t stream);
size_t dist_lds_bytes(const State& s, int pad);
size_t dist_static_lds_bytes();
int dist_max_rows();
int dist_cache_max_rows();
size_t dijkstra_lds_bytes(const State& s, int pad);
hipError_t launch_minimap(const State& s, int mini, double* out, hipStream_t stream);
__global__ void dijkstra_kernel(State s, int pad, int layer, int Lc, uint8_t* obs_out,
                                const uint32_t* list, uint32_t* count);
}  // namespace mc

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) return fail(MC_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

struct Env {
  mc_config cfg;
  double range = 0.0;
  mc_layout lay;
  mc::State s;
  int device = 0;
  int nt = 128;
  int epw = 1;  // envs per workgroup (2: two envs share one wave)
  size_t dj_lds = 0;  // dijkstra_input: LDS bytes of the BFS kernel
  uint32_t* dj_list = nullptr;  // dijkstra_input: count, done, last count + [B*N] items (full-map BFS)
  bool dj_window = true;        // dijkstra_input: window kernel first (MARLCOV_DJ_FULL=1: off)
  size_t dt_lds = 0;  // dist_reward: LDS bytes of the distance kernel
  float* dist_pre = nullptr;  // dist_reward: [B][N][8] (library-owned)
  float* dist_obs = nullptr;  // dist_reward: caller's float32 [B][N][E][E]
  double* mini_obs = nullptr; // mini_map_rad: caller's float64 [B][N][2][E][E]
  uint32_t* dist_list = nullptr;  // dist_reward: (unused), workgroups done, last count, cache hits, last hits + the shards' maps (full transform)
  uint32_t* dist_full = nullptr;  // with the cache: the split transform's list (mc_dist.hip mode 2)
  bool dist_pre_stale = true;  // dist_pre does not describe the current maps
  bool beams_set = false;
  void* beams_buf = nullptr;  // mc::Beam [beam_count]
  void* bits_buf = nullptr;   // u64 [beam_count][max(Wp, Lp)]
  void* fan_buf = nullptr;    // u32 [State::fan_words]: fan march data (dense beam sets)
  size_t fan_cap = 0;         // words allocated in fan_buf
  int beam_count = 0;
  bool grids_set = false;
  std::vector<void*> allocs;
};

struct FieldDesc {
  void* ptr;
  int64_t bytes;
};

FieldDesc field(Env* E, int f) {
  const mc::State& s = E->s;
  const int64_t B = s.B, N = s.N, mw = s.MT, G = s.G;
  switch (f) {
    case MC_FIELD_POS: return {s.pos, B * N * 2 * 4};
    case MC_FIELD_MOVED: return {s.moved, B * 8};
    case MC_FIELD_FREE: return {s.freem, B * N * mw * 8};
    case MC_FIELD_OBST: return {s.obstm, B * N * mw * 8};
    case MC_FIELD_VISITED: return {s.vis, B * mw * 8};
    case MC_FIELD_FREE_COUNT: return {s.free_cnt, B * 4};
    case MC_FIELD_VISITED_COUNT: return {s.vis_cnt, B * 4};
    case MC_FIELD_CURRSTEP: return {s.currstep, B * 4};
    case MC_FIELD_DONE_THRESH: return {s.done_thresh, B * 8};
    case MC_FIELD_ENV_GRID: return {s.env_grid, B * 4};
    case MC_FIELD_EPISODE: return {s.episode, B * 4};
    case MC_FIELD_NUMFREE: return {(void*)s.numfree, G * 4};
    case MC_FIELD_GRID_NEG: return {(void*)s.grid_neg, G * mw * 8};
    case MC_FIELD_GRID_POS: return {(void*)s.grid_pos, G * mw * 8};
    case MC_FIELD_DIST_MW: return {s.dist_mw, s.dist_mw ? B * N * 8 : -1};
    case MC_FIELD_DIST_LISTED: return {E->dist_list ? E->dist_list + 2 : nullptr, E->dist_list ? 4 : -1};
    case MC_FIELD_DIST_CACHED: return {E->dist_list ? E->dist_list + 4 : nullptr, E->dist_list ? 4 : -1};
    case MC_FIELD_EP_PC: return {s.ep_pc, B * 8};
    case MC_FIELD_EP_LEN: return {s.ep_len, B * 4};
    case MC_FIELD_DJ_LISTED: return {E->dj_list ? E->dj_list + 2 : nullptr, E->dj_list ? 4 : -1};
    case MC_FIELD_DIST_TOTALS: return {s.dist_tot, s.dist_tot ? 32 : -1};
    default: return {nullptr, -1};
  }
}

int dev_alloc(Env* E, void** p, size_t bytes) {
  void* q = nullptr;
  HIP_TRY(hipMalloc(&q, bytes < 16 ? 16 : bytes));
  HIP_TRY(hipMemset(q, 0, bytes < 16 ? 16 : bytes));
  E->allocs.push_back(q);
  *p = q;
  return MC_OK;
}

int env_threads(const mc::State& s) {
  // every lane stages at most kMaxItemsPerLane (agent, tile) items; beyond
  // that, prefer one wave per env (no cross-wave barriers) unless the beam
  // march would need more than ~8 sequential rounds per lane
  const int items = s.N * s.TW * s.TW;
  int nt = 64;
  while (nt < 1024 && items > mc::kMaxItemsPerLane * nt) nt *= 2;
  if (s.sensor == MC_SENSOR_LIDAR)
    while (nt < 256 && s.N * s.nbeams > 8 * nt) nt *= 2;
  return nt;
}

Env* as_env(void* p) { return static_cast<Env*>(p); }

// lanes per env workgroup and envs per workgroup for the current state
// (mc_create, and again when mc_set_beam_table changes the beam count)
void set_launch_shape(Env* E) {
  E->nt = env_threads(E->s);
  if (const char* ov = getenv("MARLCOV_NT")) {  // tuning / test override (64..1024)
    const int v = atoi(ov);
    if (v == 64 || v == 128 || v == 256 || v == 512 || v == 1024) E->nt = v > E->nt ? v : E->nt;
  }
  E->epw = mc::env_pack(E->s);
  if (E->nt > 64) E->epw = 1;  // (only the MARLCOV_NT override gets here with a packable env)
}

// envs per workgroup for this launch; MARLCOV_EPW=1 forces one env per
// workgroup (A/B tuning)
int launch_epw(const Env* E) {
  static const int force = [] {
    const char* v = getenv("MARLCOV_EPW");
    return v ? atoi(v) : 0;
  }();
  return force == 1 ? 1 : E->epw;
}

}  // namespace

namespace mc {
// shared with mc_super.hip: one thread-local message for mc_last_error()
void set_last_error(const char* msg) { g_err = msg; }
}  // namespace mc

extern "C" {

int32_t mc_abi_version(void) { return MARLCOV_ABI_VERSION; }

const char* mc_last_error(void) { return g_err.c_str(); }

int64_t mc_struct_size(int32_t which) {
  switch (which) {
    case 0: return (int64_t)sizeof(mc_config);
    case 1: return (int64_t)sizeof(mc_layout);
    case 2: return (int64_t)sizeof(mc_sg_config);
    case 3: return (int64_t)sizeof(mc_sg_layout);
    default: return -1;
  }
}

int64_t mc_build_param(int32_t which) {
  switch (which) {
    case MC_PARAM_DIST_CACHE_CELLS: return mc::kDistK;
    case MC_PARAM_DIST_T: return mc::kDistT;
    case MC_PARAM_DIST_MAX_ROWS: return mc::dist_max_rows();
    default: return -1;
  }
}

int mc_create(const mc_config* cfg, int hip_device, void** out_env) {
  if (!cfg || !out_env) return fail(MC_EINVAL, "mc_create: null argument");
  *out_env = nullptr;
  const mc_config& c = *cfg;
  if (c.num_envs < 1) return fail(MC_EINVAL, "num_envs must be >= 1 (got %d)", c.num_envs);
  if (c.num_agents < 1 || c.num_agents > 64)
    return fail(MC_EINVAL, "numrobot must be in [1, 64] (got %d)", c.num_agents);
  if (c.width < 3 || c.length < 3 || c.width > 32767 || c.length > 32767)
    return fail(MC_EINVAL, "padded grid %dx%d out of range", c.width, c.length);
  if (c.num_grids < 1) return fail(MC_EINVAL, "num_grids must be >= 1");
  if (c.sensor_type != MC_SENSOR_LIDAR && c.sensor_type != MC_SENSOR_SQUARE)
    return fail(MC_EINVAL, "unknown sensor_type %d", c.sensor_type);
  if (c.sensor_type == MC_SENSOR_LIDAR && c.num_beams < 1)
    return fail(MC_EINVAL, "num_lasers must be >= 1");
  if (c.sensor_type == MC_SENSOR_SQUARE && c.square_radius < 0)
    return fail(MC_EINVAL, "square sensor range must be >= 0");
  if (c.egoradius < 0) return fail(MC_EINVAL, "egoradius must be >= 0");
  if (c.pad < c.egoradius) return fail(MC_EINVAL, "pad must be >= egoradius");
  if (c.mini_map_rad < 0 || c.pad < c.mini_map_rad) return fail(MC_EINVAL, "need 0 <= mini_map_rad <= pad");
  if (c.mini_map_rad > 0 && 2 * c.egoradius + 1 > 32)
    return fail(MC_EINVAL, "minimap layers need egoradius <= 15");
  if (!(c.lidar_range == c.lidar_range)) return fail(MC_EINVAL, "lidar range is NaN");
  if (c.maxsteps < 0) return fail(MC_EINVAL, "maxsteps must be >= 0");

  int hs = 0;
  if (c.sensor_type == MC_SENSOR_LIDAR) {
    // every marked cell is within Chebyshev ceil(range) of the robot: the
    // major axis moves exactly 1 per step and the fp64 distance sum of
    // increments >= 1 reaches range after at most ceil(range) steps
    hs = c.lidar_range > 0 ? (int)ceil(c.lidar_range) : 0;
    if (c.lidar_range > 31) return fail(MC_EINVAL, "lidar range %g > 31 not supported", c.lidar_range);
  } else {
    hs = c.square_radius;
  }
  const int H = hs > c.egoradius ? hs : c.egoradius;
  const int TW = mc::window_tiles(H);
  if (2 * c.egoradius + 1 > 32)
    return fail(MC_EINVAL, "egoradius %d > 15: obs crop rows are 32-bit", c.egoradius);
  if ((int64_t)c.num_agents * TW * TW > (int64_t)mc::kMaxItemsPerLane * 1024)
    return fail(MC_EINVAL, "numrobot * %d^2 window tiles = %d exceeds %d (range/egoradius too large)",
                TW, c.num_agents * TW * TW, mc::kMaxItemsPerLane * 1024);
  {
    // the kernels index maps with 32-bit words and 24-bit factors
    const int64_t tiles = (int64_t)(((c.width + 7) / 8 + 3) / 4) * (((c.length + 7) / 8 + 3) / 4) * 16;
    if ((int64_t)c.num_envs * c.num_agents * tiles >= ((int64_t)1 << 32) ||
        (int64_t)c.num_envs * c.num_agents >= ((int64_t)1 << 24) || tiles >= ((int64_t)1 << 24))
      return fail(MC_EINVAL, "num_envs * numrobot * map tiles = %lld exceeds 2^32 words per handle",
                  (long long)c.num_envs * c.num_agents * tiles);
  }
  if (TW > mc::kMaxWindowTiles)
    return fail(MC_EINVAL, "window half-width H = %d > 27 (range/egoradius too large)", H);
  if (mc::env_lds_bytes(c.num_agents, TW, c.sensor_type == MC_SENSOR_LIDAR ? c.num_beams : 0,
                        TW <= 4 ? 4 : 8) > 65536)
    return fail(MC_EINVAL, "per-env LDS window exceeds 64 KiB (numrobot / range / num_lasers too large)");

  Env* E = new Env();
  E->cfg = c;
  E->range = c.lidar_range;
  E->device = hip_device;
  mc::State& s = E->s;
  s.B = c.num_envs;
  s.N = c.num_agents;
  s.Wp = c.width;
  s.Lp = c.length;
  s.TR = (c.width + 7) / 8;
  s.TC = (c.length + 7) / 8;
  s.TRS = (s.TR + 3) / 4;
  s.TCS = (s.TC + 3) / 4;
  s.MT = s.TRS * s.TCS * 16;
  s.G = c.num_grids;
  s.H = H;
  s.TW = TW;
  s.mg_TW = mc::magic_div((uint32_t)TW);
  s.mg_TW2 = mc::magic_div((uint32_t)(TW * TW));
  s.ego = c.egoradius;
  s.pad = c.pad;
  s.E = 2 * c.egoradius + 1;
  s.Lc = (c.mini_map_rad > 0 ? 5 : 3) + (c.dist_reward ? 1 : 0) + (c.dijkstra_input ? 1 : 0);
  s.dist = c.dist_reward ? 1 : 0;
  s.mg_LcE = mc::magic_div((uint32_t)(s.Lc * s.E));
  s.mg_E = mc::magic_div((uint32_t)s.E);
  s.sensor = c.sensor_type;
  s.nbeams = c.sensor_type == MC_SENSOR_LIDAR ? c.num_beams : 0;
  s.mg_nb = mc::magic_div((uint32_t)(s.nbeams > 0 ? s.nbeams : 1));
  s.sq_r = c.square_radius;
  s.pen = c.collision_penalty;
  s.term = c.terminal_reward;
  s.dincr = c.done_incr;
  s.maxsteps = c.maxsteps;
  s.comm_r = c.comm_radius;
  s.sst = c.single_square_tool ? 1 : 0;
  s.auto_reset = c.auto_reset ? 1 : 0;
  s.grid_mode = c.reset_grid_mode;
  s.seed = c.seed;
  s.env0 = c.env_offset;
  s.grid0 = c.grid_offset;

  hipError_t he = hipSetDevice(hip_device);
  if (he != hipSuccess) {
    delete E;
    return fail(MC_EHIP, "hipSetDevice(%d): %s", hip_device, hipGetErrorString(he));
  }
  const size_t B = s.B, N = s.N, mw = (size_t)s.MT, G = s.G;
  void* p = nullptr;
  int rc = MC_OK;
  size_t total = 0;
#define ALLOC(dst, T, count)                                  \
  do {                                                        \
    if (rc == MC_OK) rc = dev_alloc(E, &p, (count) * sizeof(T)); \
    dst = (T*)p;                                              \
    total += (count) * sizeof(T);                             \
  } while (0)
  uint64_t *gneg = nullptr, *gpos = nullptr;
  int32_t* nfree = nullptr;
  ALLOC(gneg, uint64_t, G * mw);
  ALLOC(gpos, uint64_t, G * mw);
  ALLOC(nfree, int32_t, G);
  ALLOC(s.env_grid, int32_t, B);
  ALLOC(s.pos, int32_t, B * N * 2);
  ALLOC(s.moved, uint64_t, B);
  // one extra tile past each mask array stays zero: the env kernel's staged
  // tiles outside the map read it (no select on the loaded value)
  ALLOC(s.freem, uint64_t, B * N * mw + 1);
  ALLOC(s.obstm, uint64_t, B * N * mw + 1);
  ALLOC(s.vis, uint64_t, B * mw + 1);
  ALLOC(s.free_cnt, uint32_t, B);
  ALLOC(s.vis_cnt, uint32_t, B);
  ALLOC(s.currstep, int32_t, B);
  ALLOC(s.done_thresh, double, B);
  ALLOC(s.episode, uint32_t, B);
  ALLOC(s.err, uint32_t, 4);
  ALLOC(s.ep_pc, double, B);
  ALLOC(s.ep_len, int32_t, B);
#undef ALLOC
  s.grid_neg = gneg;
  s.grid_pos = gpos;
  s.numfree = nfree;
  if (rc != MC_OK) {
    std::string msg = g_err;
    mc_destroy(E);
    return fail(rc, "%s", msg.c_str());
  }
  {
    std::vector<int32_t> eg(B);
    for (size_t i = 0; i < B; ++i) eg[i] = (int32_t)(i % G);
    std::vector<double> dt(B, c.done_thresh);
    if (hipMemcpy(s.env_grid, eg.data(), B * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s.done_thresh, dt.data(), B * 8, hipMemcpyHostToDevice) != hipSuccess) {
      mc_destroy(E);
      return fail(MC_EHIP, "mc_create: initial upload failed");
    }
  }
  set_launch_shape(E);
  if (c.dijkstra_input) {
    // the BFS bitboards of one (env, agent) live in one workgroup's LDS
    const size_t need = mc::dijkstra_lds_bytes(s, c.pad);
    int maxlds = 0;
    if (hipDeviceGetAttribute(&maxlds, hipDeviceAttributeMaxSharedMemoryPerBlock, hip_device) !=
            hipSuccess ||
        need + 1024 > (size_t)maxlds) {
      mc_destroy(E);
      return fail(MC_EINVAL, "dijkstra_input: %zu B of LDS bitboards for a %dx%d grid exceed the "
                  "device's %d B per workgroup", need, c.width, c.length, maxlds);
    }
    E->dj_lds = need;
    void* lq = nullptr;
    if (dev_alloc(E, &lq, ((size_t)s.B * s.N + 3) * 4) != MC_OK) {
      std::string msg = g_err;
      mc_destroy(E);
      return fail(MC_EHIP, "dijkstra_input state: %s", msg.c_str());
    }
    E->dj_list = (uint32_t*)lq;
    const char* fo = getenv("MARLCOV_DJ_FULL");  // parity tests: every item on the full map
    E->dj_window = !(fo && atoi(fo) == 1);
  }
  if (c.dist_reward) {
    if (c.width + c.length + 4 * c.pad >= 65535) {
      mc_destroy(E);
      return fail(MC_EINVAL, "dist_reward: grid %dx%d too large for 16-bit distances", c.width,
                  c.length);
    }
    if (s.Wp + 2 * c.pad > mc::dist_max_rows()) {
      mc_destroy(E);
      return fail(MC_EINVAL, "dist_reward: %d extended rows exceed the transform's %d", s.Wp + 2 * c.pad,
                  mc::dist_max_rows());
    }
    if (s.Lp + 2 * c.pad > 32767) {  // the witness column is a signed 16-bit half (mc_device.h)
      mc_destroy(E);
      return fail(MC_EINVAL, "dist_reward: %d extended columns exceed 32767", s.Lp + 2 * c.pad);
    }
    const size_t need = mc::dist_lds_bytes(s, c.pad);
    int maxlds = 0;
    if (hipDeviceGetAttribute(&maxlds, hipDeviceAttributeMaxSharedMemoryPerBlock, hip_device) !=
            hipSuccess ||
        need + mc::dist_static_lds_bytes() + 1024 > (size_t)maxlds) {
      mc_destroy(E);
      return fail(MC_EINVAL, "dist_reward: %zu B of LDS bitboards for a %dx%d grid exceed the "
                  "device's %d B per workgroup", need, c.width, c.length, maxlds);
    }
    E->dt_lds = need;
    void* q = nullptr;
    if (dev_alloc(E, &q, (size_t)s.B * s.N * 8 * sizeof(float)) != MC_OK) {
      std::string msg = g_err;
      mc_destroy(E);
      return fail(MC_EHIP, "%s", msg.c_str());
    }
    E->dist_pre = (float*)q;
    E->s.dist_pre = E->dist_pre;
    // (M, witness) per map, M = -1 (unknown) until a full transform; the
    // work list of the full transform and its count
    void *mw = nullptr, *lq = nullptr, *tq = nullptr, *sh = nullptr;
    const size_t cap = (size_t)((s.B + mc::kListShards - 1) / mc::kListShards) * s.N;  // entries per shard
    if (dev_alloc(E, &mw, (size_t)s.B * s.N * 8) != MC_OK ||
        dev_alloc(E, &lq, (mc::kListShards * cap + 5) * 4) != MC_OK || dev_alloc(E, &tq, 32) != MC_OK ||
        dev_alloc(E, &sh, mc::kListShards * mc::kShardStride * 4) != MC_OK ||
        hipMemset(mw, 0xFF, (size_t)s.B * s.N * 8) != hipSuccess) {
      std::string msg = g_err;
      mc_destroy(E);
      return fail(MC_EHIP, "dist_reward state: %s", msg.c_str());
    }
    E->s.dist_mw = (int32_t*)mw;
    E->dist_list = (uint32_t*)lq;
    E->s.dist_cnt = E->dist_list;
    E->s.dist_shc = (uint32_t*)sh;
    E->s.dist_cap = (uint32_t)cap;
    E->s.dist_tot = (unsigned long long*)tq;
    // the top-cell cache (mc_dist.hip), off with map sharing (other agents'
    // maps add cells outside the agent's own sensing windows) or
    // MARLCOV_DIST_CACHE=0
    const char* dc = getenv("MARLCOV_DIST_CACHE");
    // and off for maps past the LDS-bitboard transform's rows (the big-map
    // kernel transforms every listed map whole, mc_dist.hip)
    if (!c.map_sharing && !(dc && dc[0] == '0') && s.Wp + 2 * c.pad <= mc::dist_cache_max_rows()) {
      void *cc = nullptr, *cd = nullptr, *ch = nullptr, *sm = nullptr;
      void *gk = nullptr, *gc = nullptr, *ga = nullptr, *fl = nullptr, *pc = nullptr, *rm = nullptr, *go = nullptr;
      const size_t maps = (size_t)s.B * s.N;
      if (dev_alloc(E, &cc, maps * mc::kDistK * 4) != MC_OK || dev_alloc(E, &cd, maps * mc::kDistK * 4) != MC_OK ||
          dev_alloc(E, &ch, maps * 32) != MC_OK || hipMemset(ch, 0xFF, maps * 32) != hipSuccess ||
          dev_alloc(E, &sm, maps * mc::kDistStrips * 4) != MC_OK || dev_alloc(E, &gk, maps * 8) != MC_OK ||
          dev_alloc(E, &gc, (size_t)mc::kDistGSlots * mc::kDistGParts * 4) != MC_OK || dev_alloc(E, &pc, maps * 4) != MC_OK ||
          dev_alloc(E, &go, (size_t)mc::kDistGSlots * 4) != MC_OK ||
          dev_alloc(E, &rm, maps * 8) != MC_OK ||
          dev_alloc(E, &ga, (size_t)mc::kDistGSlots * mc::kDistGParts * mc::kDistK * 8) != MC_OK ||
          dev_alloc(E, &fl, (maps * 2 + 8) * 4) != MC_OK) {
        std::string msg = g_err;
        mc_destroy(E);
        return fail(MC_EHIP, "dist_reward cache: %s", msg.c_str());
      }
      E->s.dist_cc = (int32_t*)cc;
      E->s.dist_cd = (int32_t*)cd;
      E->s.dist_ch = (int32_t*)ch;
      E->s.dist_sm = (uint32_t*)sm;
      E->s.dist_pcnt = (uint32_t*)pc;
      E->s.dist_rmask = (unsigned long long*)rm;
      E->s.dist_gkey = (unsigned long long*)gk;
      E->s.dist_gcnt = (uint32_t*)gc;
      E->s.dist_govf = (uint32_t*)go;
      E->s.dist_gcand = (int2*)ga;
      // MARLCOV_DIST_SPLIT=0: every listed map's full transform in one workgroup
      const char* sp = getenv("MARLCOV_DIST_SPLIT");
      if (!(sp && sp[0] == '0')) E->dist_full = E->s.dist_full = (uint32_t*)fl;
    }
  }
  mc_layout& L = E->lay;
  L.tile_rows = 4 * s.TRS;
  L.tile_cols = 4 * s.TCS;
  L.window_half = s.H;
  L.window_tiles = s.TW;
  L.obs_layers = s.Lc;
  L.obs_side = s.E;
  L.obs_bytes_per_env = (int64_t)N * s.Lc * s.E * s.E;
  L.mask_words_per_agent = (int64_t)mw;
  L.state_bytes = (int64_t)total;
  if (s.sensor != MC_SENSOR_LIDAR) E->beams_set = true;
  *out_env = E;
  return MC_OK;
}

void mc_destroy(void* env) {
  Env* E = as_env(env);
  if (!E) return;
  (void)hipSetDevice(E->device);
  for (void* p : E->allocs) (void)hipFree(p);
  if (E->beams_buf) (void)hipFree(E->beams_buf);
  if (E->bits_buf) (void)hipFree(E->bits_buf);
  if (E->fan_buf) (void)hipFree(E->fan_buf);
  delete E;
}

int mc_query(void* env, mc_layout* out) {
  if (!env || !out) return fail(MC_EINVAL, "mc_query: null argument");
  *out = as_env(env)->lay;
  return MC_OK;
}

// Fan march data of a dense beam set (mc_env_kernel.hip fan_march, layout in
// mc_internal.h State::fan_data).  Beams are grouped by octant class (major
// axis, major sign, minor sign; minor sign 0 counts as +), ordered by their
// minor offsets, and cut greedily into sectors of up to kFanS beams whose
// offsets differ by 0 or 1 between neighbours at every step, at most one
// start-dependent beam (Beam::axis bit 1) per sector.  The two classes of a
// line (same major axis and sign, minor sign + / -) are paired: sector i of
// each, interleaved step by step in one pair record (an empty sector pads the
// shorter class), so one lane reads the line word once for both and marks it
// with one OR; the pairs of the four lines are interleaved, so the pairs of
// one march instruction mark different lines.
// A start-dependent beam marches with its common bits except from the minor
// starts where its own bits differ before the march ends (bits[b][start],
// cm starts); the kernel marches those alone.  Returns false (ray march) for
// sparse sets: fewer than 64 beams (dense_beams), or fewer than two beams per
// sector on average.
static bool build_fan(const std::vector<mc::Beam>& bt, const std::vector<uint64_t>& bits, int cmax, int Wp,
                      int Lp, int kmax, int N, int lanes, std::vector<uint32_t>& out, int& nsec, int& nspec) {
  const int nb = (int)bt.size();
  if (nb < 64 || kmax > 27) return false;
  auto off = [](const mc::Beam& o, int k) {  // signed minor offset of step k
    return o.msign * __builtin_popcount(o.bits & ((1u << k) - 1u));
  };
  std::vector<std::vector<int>> cls(8);
  std::vector<int> spec;
  for (int b = 0; b < nb; ++b) {
    const mc::Beam& o = bt[b];
    if (o.axis & 2) spec.push_back(b);
    cls[(o.axis & 1) * 4 + (o.sign < 0 ? 2 : 0) + (o.msign < 0 ? 1 : 0)].push_back(b);
  }
  std::vector<std::vector<std::vector<int>>> secs(8);
  size_t most = 0;
  for (int c = 0; c < 8; ++c) {
    std::vector<int>& v = cls[c];
    std::sort(v.begin(), v.end(), [&](int p, int q) {
      for (int k = kmax; k >= 1; --k) {
        const int a = off(bt[p], k), d = off(bt[q], k);
        if (a != d) return a < d;
      }
      return p < q;
    });
    for (int b : v) {
      std::vector<std::vector<int>>& S = secs[c];
      bool join = !S.empty() && (int)S.back().size() < mc::kFanS;
      if (join && (bt[b].axis & 2))
        for (int o : S.back()) join = join && !(bt[o].axis & 2);
      for (int k = 1; join && k <= kmax; ++k) {
        const int d = off(bt[b], k) - off(bt[S.back().back()], k);
        join = d == 0 || d == 1;
      }
      if (join) S.back().push_back(b);
      else S.push_back({b});
    }
    most = std::max(most, secs[c].size());
  }
  static const std::vector<int> kNone;
  std::vector<std::pair<const std::vector<int>*, const std::vector<int>*>> order;  // (minor +, minor -)
  int real = 0;
  for (size_t i = 0; i < most; ++i)
    for (int m = 0; m < 4; ++m) {
      const bool p = i < secs[2 * m].size(), q = i < secs[2 * m + 1].size();
      if (p || q) order.push_back({p ? &secs[2 * m][i] : &kNone, q ? &secs[2 * m + 1][i] : &kNone});
      real += (int)p + (int)q;
    }
  nsec = 2 * (int)order.size();  // sector slots (pairs x 2, empty ones included)
  nspec = (int)spec.size();
  if (2 * real > nb || N * nspec > lanes || nspec > 255) return false;
  out.assign(mc::kFanLutBytes / 4, 0u);
  uint8_t* lut = reinterpret_cast<uint8_t*>(out.data());
  for (int D = 0; D < 32; ++D) {
    int r[mc::kFanS] = {0};  // cell of beam i
    for (int i = 1; i < mc::kFanS; ++i) r[i] = r[i - 1] + ((D >> (i - 1)) & 1);
    for (int A = 0; A < 64; ++A) {
      int lit = 0, kill = 0;
      for (int i = 0; i < mc::kFanS; ++i) {
        if ((A >> i) & 1) lit |= 1 << r[i];      // spread: beams A -> their cells
        if ((A >> r[i]) & 1) kill |= 1 << i;     // expand: cells A -> the beams on them
      }
      lut[D * 64 + A] = (uint8_t)lit;
      lut[2048 + D * 64 + A] = (uint8_t)kill;
    }
  }
  auto cbits = [](const mc::Beam& o) {
    return ((o.axis & 1) ? (uint32_t)mc::FAN_COLS : 0u) | (o.sign < 0 ? (uint32_t)mc::FAN_NEG : 0u);
  };
  // word 0 of a sector: its class bits and special beam; word k: step k's
  // entry (an empty sector: the partner's class bits, entries 0 = no beam)
  auto desc = [&](const std::vector<int>& v, uint32_t cls) {
    uint32_t w0 = v.empty() ? cls : cbits(bt[v[0]]);
    for (size_t j = 0; j < v.size(); ++j)
      if (bt[v[j]].axis & 2) {
        const size_t si = std::find(spec.begin(), spec.end(), v[j]) - spec.begin();
        w0 |= mc::FAN_SPECIAL | ((uint32_t)j << 3) | ((uint32_t)si << 8);
      }
    return w0;
  };
  auto entry = [&](const std::vector<int>& v, int k) {
    if (v.empty()) return 0u;
    const int lo = off(bt[v[0]], k);
    uint32_t D = 0, valid = 0;
    for (size_t j = 0; j < v.size(); ++j) {
      if (j + 1 < v.size() && off(bt[v[j + 1]], k) != off(bt[v[j]], k)) D |= 1u << j;
      if (bt[v[j]].K >= k) valid |= 1u << j;
    }
    return (uint32_t)(lo + 32) | (D << 6) | (valid << 16);
  };
  for (const auto& pr : order) {  // pair record: [desc+, desc-], then [entry+(k), entry-(k)] per step
    const std::vector<int>& v0 = *pr.first;
    const std::vector<int>& v1 = *pr.second;
    const uint32_t cls = cbits(bt[(v0.empty() ? v1 : v0)[0]]);
    out.push_back(desc(v0, cls));
    out.push_back(desc(v1, cls));
    for (int k = 1; k <= kmax; ++k) {
      out.push_back(entry(v0, k));
      out.push_back(entry(v1, k));
    }
  }
  for (int b : spec) {
    // the starts whose own bits leave the common path before the march ends
    // (the check of mc_set_beam_table's common-pattern test)
    const mc::Beam& o = bt[b];
    const int cm = (o.axis & 1) == 0 ? Lp : Wp;
    const uint64_t* row = &bits[(size_t)b * cmax];
    int elo = 1 << 30, ehi = -1;
    for (int c0 = 1; c0 + 1 < cm; ++c0) {
      int p = c0, c = c0;
      for (int k = 0; k < o.K; ++k) {
        p += ((row[c0] >> k) & 1) ? o.msign : 0;
        c += ((o.bits >> k) & 1) ? o.msign : 0;
        if (p != c) { elo = std::min(elo, c0); ehi = std::max(ehi, c0); break; }
        if (p <= 0 || p >= cm - 1) break;
      }
    }
    const uint32_t rec[8] = {(uint32_t)b, cbits(o), (uint32_t)o.msign, (uint32_t)o.K,
                             (uint32_t)elo, (uint32_t)ehi, 0u, 0u};
    out.insert(out.end(), rec, rec + 8);
  }
  while (out.size() % 4) out.push_back(0u);
  return true;
}

int mc_set_beam_table(void* env, const double* host_table, int32_t num_beams) {
  Env* E = as_env(env);
  if (!E || !host_table) return fail(MC_EINVAL, "mc_set_beam_table: null argument");
  if (E->s.sensor != MC_SENSOR_LIDAR) return fail(MC_EINVAL, "beam table on a non-lidar env");
  if (num_beams < 1) return fail(MC_EINVAL, "beam table needs >= 1 beam");
  // the per-env LDS budget mc_create checked holds 16 B per beam: a new beam
  // count must fit it too, or the next launch would fail inside HIP
  if (mc::env_lds_bytes(E->s.N, E->s.TW, num_beams, E->s.TW <= 4 ? 4 : 8) > 65536)
    return fail(MC_EINVAL, "mc_set_beam_table: %d beams exceed the 64 KiB per-env LDS window", num_beams);
  const int cmax = E->s.Wp > E->s.Lp ? E->s.Wp : E->s.Lp;
  std::vector<mc::Beam> bt(num_beams);
  std::vector<uint64_t> bits((size_t)num_beams * cmax, 0);
  int kmax = 0, kmin = 1 << 30;
  bool common = true;
  for (int b = 0; b < num_beams; ++b) {
    const double xi = host_table[3 * b], yi = host_table[3 * b + 1], di = host_table[3 * b + 2];
    mc::Beam& o = bt[b];
    double minor;
    // lidar.py:43-45 normalises by max(|xinc|, |yinc|): one of them is +-1
    if (fabs(xi) == 1.0 && fabs(yi) <= 1.0) {
      o.axis = 0; o.sign = xi > 0 ? 1 : -1; minor = yi;
    } else if (fabs(yi) == 1.0 && fabs(xi) <= 1.0) {
      o.axis = 1; o.sign = yi > 0 ? 1 : -1; minor = xi;
    } else {
      return fail(MC_EINVAL, "beam %d is not a normalised lidar.py increment (%g, %g)", b, xi, yi);
    }
    o.msign = minor > 0 ? 1 : (minor < 0 ? -1 : 0);
    o.bits = 0;
    if (!(di >= 1.0)) return fail(MC_EINVAL, "beam %d distinc %g < 1", b, di);
    // currdist = 0; while currdist < range: currdist += distinc  (lidar.py:49-56)
    double dist = 0.0;
    int K = 0;
    while (dist < E->range && K <= 64) { dist += di; ++K; }
    if (K > E->s.H)
      return fail(MC_EINVAL, "beam %d takes %d steps > window half-width %d", b, K, E->s.H);
    o.K = K;
    kmax = K > kmax ? K : kmax;
    kmin = K < kmin ? K : kmin;
    // the reference's minor-coordinate chain (currx/curry += inc, int() of it)
    // from every integer start; valid starts are the padded-grid interior
    const int cm = o.axis == 0 ? E->s.Lp : E->s.Wp;
    for (int c0 = 0; c0 < cm; ++c0) {
      double m = (double)c0;
      int cell = c0;
      uint64_t w = 0;
      for (int k = 0; k < K; ++k) {
        m += minor;
        const int next = (int)m;  // trunc toward zero, as Python int()
        const int d = next - cell;
        if (d != 0 && d != o.msign) {
          if (m >= 0.0)  // negative coordinates lie outside the grid: unused
            return fail(MC_EINVAL, "beam %d start %d: minor step %d at k=%d", b, c0, d, k);
        }
        if (d != 0) w |= 1ull << k;
        cell = next;
      }
      bits[(size_t)b * cmax + c0] = w;
    }
    // the pattern of most starts; it stands for the beam's table when every
    // start a robot can occupy (1 .. cm-2: the border is -1) visits the same
    // cells with it up to the first border cell of the minor axis, where the
    // march ends (an obstacle) -- then the rest of the word is never read.
    // A beam without such a pattern is flagged (axis bit 1) and marches from
    // its per-start table (C4's 360 beams: 2 of them, 270 and 315 degrees,
    // whose float64 chains truncate differently at starts 1..3)
    {
      bool bc = true;
      const uint64_t* row = &bits[(size_t)b * cmax];
      uint64_t best = row[cm > 2 ? 1 : 0];
      int best_n = 0;
      for (int c0 = 1; c0 + 1 < cm; ++c0) {
        int n = 0;
        for (int c1 = 1; c1 + 1 < cm; ++c1) n += row[c1] == row[c0];
        if (n > best_n) { best_n = n; best = row[c0]; }
        if (2 * n > cm) break;
      }
      o.bits = (uint32_t)best;
      for (int c0 = 1; c0 + 1 < cm && bc; ++c0) {
        int a = c0, c = c0;  // cell of the start's own word / of the common word
        for (int k = 0; k < K; ++k) {
          a += ((row[c0] >> k) & 1) ? o.msign : 0;
          c += ((best >> k) & 1) ? o.msign : 0;
          if (a != c) { bc = false; break; }
          if (a <= 0 || a >= cm - 1) break;  // border reached: the march ends here
        }
      }
      if (!bc) o.axis |= 2;
      common = common && bc;
    }
  }
  HIP_TRY(hipSetDevice(E->device));
  // a queued launch (on any stream) may still read the tables: let it finish
  // before they are overwritten or freed.  Until the new tables are complete
  // the handle has none (a failure below leaves mc_step refusing to run
  // rather than reading freed or half-written tables).
  HIP_TRY(hipDeviceSynchronize());
  E->beams_set = false;
  E->s.fan_nsec = E->s.fan_nspec = E->s.fan_kt = E->s.fan_words = 0;
  E->s.fan_data = nullptr;
  if (num_beams != E->beam_count || !E->beams_buf) {
    // the reference lets callers swap _thetalist after construction
    // (even beam counts): (re-)size the device tables
    E->beam_count = 0;
    if (E->beams_buf) (void)hipFree(E->beams_buf);
    if (E->bits_buf) (void)hipFree(E->bits_buf);
    E->beams_buf = E->bits_buf = nullptr;
    HIP_TRY(hipMalloc(&E->beams_buf, (size_t)num_beams * sizeof(mc::Beam)));
    HIP_TRY(hipMalloc(&E->bits_buf, bits.size() * sizeof(uint64_t)));
    E->beam_count = num_beams;
    E->s.beams = (const mc::Beam*)E->beams_buf;
    E->s.beam_bits = (const uint64_t*)E->bits_buf;
    E->s.bcmax = cmax;
    E->s.nbeams = num_beams;
    E->s.mg_nb = mc::magic_div((uint32_t)num_beams);
    E->cfg.num_beams = num_beams;
    set_launch_shape(E);
  }
  HIP_TRY(hipMemcpy((void*)E->s.beams, bt.data(), (size_t)num_beams * sizeof(mc::Beam),
                    hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy((void*)E->s.beam_bits, bits.data(), bits.size() * sizeof(uint64_t),
                    hipMemcpyHostToDevice));
  E->s.beam_kmax = kmax;
  E->s.beam_kmin = kmin;
  E->s.beam_common = common && !getenv("MARLCOV_BEAM_TABLE") ? 1 : 0;
  // step-1 cells of the common patterns (lidar.py:52-56: every beam with
  // K >= 1 reaches its step-1 cell from the free robot cell)
  uint32_t k1 = 1u << 4;  // the robot cell (step 0)
  for (int b = 0; b < num_beams; ++b) {
    const mc::Beam& o = bt[b];
    if (o.K < 1) continue;
    const int mv = (o.bits & 1u) ? o.msign : 0;
    const int dx = (o.axis & 1) == 0 ? o.sign : mv, dy = (o.axis & 1) == 0 ? mv : o.sign;
    k1 |= 1u << (3 * (dx + 1) + (dy + 1));
  }
  E->s.beam_k1 = E->s.beam_common && !getenv("MARLCOV_NO_K1") ? k1 : 0u;
  // fan march of a dense set (after nt / epw: they bound the special lanes);
  // MARLCOV_FAN=0 or MARLCOV_BEAM_TABLE keep the ray march (parity A/B)
  {
    std::vector<uint32_t> fd;
    int nsec = 0, nspec = 0;
    const char* fv = getenv("MARLCOV_FAN");
    bool on = !getenv("MARLCOV_BEAM_TABLE") && !(fv && fv[0] == '0') &&
              build_fan(bt, bits, cmax, E->s.Wp, E->s.Lp, kmax, E->s.N, E->nt / E->epw, fd, nsec, nspec);
    const int rb = E->s.TW <= 4 ? 4 : 8;
    if (on && mc::env_lds_bytes(E->s.N, E->s.TW, num_beams, rb,
                                mc::fan_lds_bytes(E->s.N, nspec, kmax, (int)fd.size())) > 65536)
      on = false;
    if (on) {
      if (fd.size() > E->fan_cap) {
        if (E->fan_buf) (void)hipFree(E->fan_buf);
        E->fan_buf = nullptr;
        E->fan_cap = 0;
        HIP_TRY(hipMalloc(&E->fan_buf, fd.size() * 4));
        E->fan_cap = fd.size();
      }
      HIP_TRY(hipMemcpy(E->fan_buf, fd.data(), fd.size() * 4, hipMemcpyHostToDevice));
      E->s.fan_data = (const uint32_t*)E->fan_buf;
      E->s.fan_nsec = nsec;
      E->s.fan_nspec = nspec;
      E->s.fan_kt = kmax;
      E->s.fan_words = (int)fd.size();
    }
  }
  E->beams_set = true;
  return MC_OK;
}

static int check_numfree(Env* E, hipStream_t st) {
  std::vector<int32_t> nf(E->s.G);
  HIP_TRY(hipMemcpyAsync(nf.data(), E->s.numfree, nf.size() * 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  for (int g = 0; g < E->s.G; ++g)
    if (nf[g] <= 0)
      return fail(MC_EINVAL,
                  "grid %d has no cell > 0: the reference's percent_covered() divides by "
                  "count_nonzero(grid > 0) (dec_grid_rl.py:552)",
                  g);
  E->grids_set = true;
  return MC_OK;
}

int mc_set_grids(void* env, const int8_t* dev_grids, int32_t num_grids, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_grids) return fail(MC_EINVAL, "mc_set_grids: null argument");
  if (num_grids != E->s.G)
    return fail(MC_EINVAL, "mc_set_grids: %d grids, config says %d", num_grids, E->s.G);
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMemsetAsync((void*)E->s.numfree, 0, (size_t)E->s.G * 4, st));
  HIP_TRY(mc::launch_pack(E->s, dev_grids, st));
  return check_numfree(E, st);
}

int mc_generate_grids(void* env, uint64_t seed, double p_obst, void* stream) {
  Env* E = as_env(env);
  if (!E) return fail(MC_EINVAL, "mc_generate_grids: null env");
  if (!(p_obst >= 0.0 && p_obst < 1.0)) return fail(MC_EINVAL, "p_obst must be in [0, 1)");
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMemsetAsync((void*)E->s.numfree, 0, (size_t)E->s.G * 4, st));
  HIP_TRY(mc::launch_gen(E->s, seed, p_obst, st));
  return check_numfree(E, st);
}

int mc_random_actions(void* env, uint64_t seed, int32_t step, uint8_t* dev_actions, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_actions) return fail(MC_EINVAL, "mc_random_actions: null argument");
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(mc::launch_random_actions(E->s, seed, step, dev_actions, (hipStream_t)stream));
  return MC_OK;
}

const char* mc_kernel_variant(void* env) {
  Env* E = as_env(env);
  if (!E) {
    fail(MC_EINVAL, "mc_kernel_variant: null env");
    return "";
  }
  // the lidar's march: "+fan(S/P)" = fan_march over S sectors and P special
  // beams (dense beam sets), else the ray march
  thread_local std::string name;
  name = mc::env_variant(E->s, E->nt, launch_epw(E));
  if (E->s.sensor == MC_SENSOR_LIDAR && E->s.fan_nsec + E->s.fan_nspec > 0)
    name += " +fan(" + std::to_string(E->s.fan_nsec) + "/" + std::to_string(E->s.fan_nspec) + ")";
  return name.c_str();
}

int mc_set_env_grids(void* env, const int32_t* dev_env_grid, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_env_grid) return fail(MC_EINVAL, "mc_set_env_grids: null argument");
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMemcpyAsync(E->s.env_grid, dev_env_grid, (size_t)E->s.B * 4, hipMemcpyDeviceToDevice,
                         (hipStream_t)stream));
  return MC_OK;
}

// dijkstra_input: obs layer 3 from the post-step maps (dec_grid_rl.py:354-358),
// a second kernel on the same stream
static int dijkstra_layer(Env* E, void* dev_obs, hipStream_t st) {
  if (E->cfg.mini_map_rad > 0) {  // the minimap overwrites layer 3 (dec_grid_rl.py:365)
    HIP_TRY(mc::launch_minimap(E->s, E->cfg.mini_map_rad, E->mini_obs, st));
    return MC_OK;
  }
  if (!E->cfg.dijkstra_input) return MC_OK;
  if (E->dj_lds > 65536)
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(&mc::dijkstra_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)E->dj_lds));
  HIP_TRY(mc::launch_dijkstra(E->s, E->cfg.pad, 3, E->s.Lc, (uint8_t*)dev_obs, E->dj_list,
                              E->dj_window, st));
  return MC_OK;
}

// dist_reward: the distance terms of the maps before sensing (PRE, read by
// the env kernel's reward) or the obs layer of the maps after it (POST)
static int dist_terms(Env* E, int post, hipStream_t st) {
  if (!E->cfg.dist_reward) return MC_OK;
  if (post)  // the full transform of the maps the env kernel listed (unknown max(d), or a
             // target its window search could not settle)
    HIP_TRY(mc::launch_dist_listed(E->s, E->cfg.pad, E->dist_pre, E->dist_obs, E->dist_list + 5,
                                   E->dist_list, E->dist_full, st));
  else
    HIP_TRY(mc::launch_dist(E->s, E->cfg.pad, 0, E->dist_pre, E->dist_obs, st));
  E->dist_pre_stale = !post;  // a POST transform leaves PRE data for the next step
  return MC_OK;
}

static int ready(Env* E, const char* who) {
  if (!E->beams_set) return fail(MC_ESTATE, "%s: lidar beam table not set (mc_set_beam_table)", who);
  if (!E->grids_set) return fail(MC_ESTATE, "%s: grids not set (mc_set_grids / mc_generate_grids)", who);
  if (E->cfg.dist_reward && !E->dist_obs)
    return fail(MC_ESTATE, "%s: dist_reward needs the float obs buffer (mc_set_dist_obs)", who);
  if (E->cfg.mini_map_rad > 0 && !E->mini_obs)
    return fail(MC_ESTATE, "%s: mini_map_rad needs the float64 minimap buffer (mc_set_minimap_obs)", who);
  return MC_OK;
}

int mc_reset(void* env, const uint8_t* dev_env_mask, const int32_t* dev_pos, void* dev_obs,
             uint8_t* dev_adj, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_obs) return fail(MC_EINVAL, "mc_reset: null argument");
  int rc = ready(E, "mc_reset");
  if (rc) return rc;
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(mc::launch_env(E->s, mc::MODE_RESET, nullptr, dev_env_mask, dev_pos, nullptr, nullptr,
                         (uint8_t*)dev_obs, dev_adj, E->nt, launch_epw(E), (hipStream_t)stream));
  rc = dijkstra_layer(E, dev_obs, (hipStream_t)stream);
  if (rc) return rc;
  return dist_terms(E, 1, (hipStream_t)stream);
}

// the launches of one step (the caller checked the arguments and set the device)
static int step_once(Env* E, const uint8_t* dev_actions, double* dev_reward, uint8_t* dev_done,
                     void* dev_obs, uint8_t* dev_adj, hipStream_t st) {
  int rc;
  if (E->cfg.map_sharing) HIP_TRY(mc::launch_share(E->s, dev_actions, st));
  if (E->cfg.map_sharing || E->dist_pre_stale) {
    rc = dist_terms(E, 0, st);  // observe() reads the maps before sensing
    if (rc) return rc;
  }
  HIP_TRY(mc::launch_env(E->s, mc::MODE_STEP, dev_actions, nullptr, nullptr, dev_reward, dev_done,
                         (uint8_t*)dev_obs, dev_adj, E->nt, launch_epw(E), st));
  rc = dijkstra_layer(E, dev_obs, st);
  if (rc) return rc;
  return dist_terms(E, 1, st);
}

int mc_step(void* env, const uint8_t* dev_actions, double* dev_reward, uint8_t* dev_done,
            void* dev_obs, uint8_t* dev_adj, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_actions || !dev_reward || !dev_done || !dev_obs)
    return fail(MC_EINVAL, "mc_step: null argument");
  int rc = ready(E, "mc_step");
  if (rc) return rc;
  HIP_TRY(hipSetDevice(E->device));
  return step_once(E, dev_actions, dev_reward, dev_done, dev_obs, dev_adj, (hipStream_t)stream);
}

int mc_step_many(void* env, const uint8_t* dev_actions, int64_t actions_stride, int32_t num_steps,
                 double* dev_reward, int64_t reward_stride, uint8_t* dev_done, int64_t done_stride,
                 void* dev_obs, int64_t obs_stride, uint8_t* dev_adj, int64_t adj_stride, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_actions || !dev_reward || !dev_done || !dev_obs)
    return fail(MC_EINVAL, "mc_step_many: null argument");
  if (num_steps < 0 || actions_stride < 0 || reward_stride < 0 || done_stride < 0 || obs_stride < 0 ||
      adj_stride < 0)
    return fail(MC_EINVAL, "mc_step_many: negative step count or stride");
  if (reward_stride % 8 != 0) return fail(MC_EINVAL, "mc_step_many: reward_stride must be a multiple of 8 bytes");
  int rc = ready(E, "mc_step_many");
  if (rc) return rc;
  HIP_TRY(hipSetDevice(E->device));
  hipStream_t st = (hipStream_t)stream;
  for (int32_t k = 0; k < num_steps; ++k) {
    rc = step_once(E, dev_actions + k * actions_stride,
                   reinterpret_cast<double*>(reinterpret_cast<char*>(dev_reward) + k * reward_stride),
                   dev_done + k * done_stride, static_cast<char*>(dev_obs) + k * obs_stride,
                   dev_adj ? dev_adj + k * adj_stride : nullptr, st);
    if (rc) {  // steps 0..k-1 are enqueued: the env has advanced k steps
      std::string msg = g_err;
      return fail(rc, "mc_step_many: step %d of %d failed after %d steps were enqueued: %s", (int)k,
                  (int)num_steps, (int)k, msg.c_str());
    }
  }
  return MC_OK;
}

int64_t mc_field_bytes(void* env, int32_t f) {
  Env* E = as_env(env);
  if (!E) return fail(MC_EINVAL, "mc_field_bytes: null env");
  FieldDesc d = field(E, f);
  if (!d.ptr) return fail(MC_EINVAL, "unknown state field %d", f);
  return d.bytes;
}

int mc_get_state(void* env, int32_t f, void* dev_dst, int64_t bytes, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_dst) return fail(MC_EINVAL, "mc_get_state: null argument");
  FieldDesc d = field(E, f);
  if (!d.ptr) return fail(MC_EINVAL, "unknown state field %d", f);
  if (bytes != d.bytes) return fail(MC_EINVAL, "field %d is %lld bytes, got %lld", f, (long long)d.bytes, (long long)bytes);
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMemcpyAsync(dev_dst, d.ptr, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return MC_OK;
}

int mc_set_state(void* env, int32_t f, const void* dev_src, int64_t bytes, void* stream) {
  Env* E = as_env(env);
  if (!E || !dev_src) return fail(MC_EINVAL, "mc_set_state: null argument");
  FieldDesc d = field(E, f);
  if (!d.ptr) return fail(MC_EINVAL, "unknown state field %d", f);
  if (f == MC_FIELD_DIST_MW || f == MC_FIELD_DIST_LISTED || f == MC_FIELD_EP_PC || f == MC_FIELD_EP_LEN ||
      f == MC_FIELD_DJ_LISTED || f == MC_FIELD_DIST_CACHED || f == MC_FIELD_DIST_TOTALS)
    return fail(MC_EINVAL, "field %d is derived state (read-only)", f);
  if (bytes != d.bytes) return fail(MC_EINVAL, "field %d is %lld bytes, got %lld", f, (long long)d.bytes, (long long)bytes);
  HIP_TRY(hipSetDevice(E->device));
  HIP_TRY(hipMemcpyAsync(d.ptr, dev_src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  if (f == MC_FIELD_GRID_NEG || f == MC_FIELD_GRID_POS || f == MC_FIELD_NUMFREE) E->grids_set = true;
  E->dist_pre_stale = true;  // uploaded maps / positions: recompute the PRE terms
  if (E->s.dist_mw)  // and max(d) of every map
    HIP_TRY(hipMemsetAsync(E->s.dist_mw, 0xFF, (size_t)E->s.B * E->s.N * 8, (hipStream_t)stream));
  if (E->s.dist_ch)  // and the top-cell caches
    HIP_TRY(hipMemsetAsync(E->s.dist_ch, 0xFF, (size_t)E->s.B * E->s.N * 32, (hipStream_t)stream));
  return MC_OK;
}

int mc_set_dist_obs(void* env, float* dev_dist_obs) {
  Env* E = as_env(env);
  if (!E || !dev_dist_obs) return fail(MC_EINVAL, "mc_set_dist_obs: null argument");
  if (!E->cfg.dist_reward) return fail(MC_EINVAL, "mc_set_dist_obs: config has dist_reward = 0");
  E->dist_obs = dev_dist_obs;
  E->s.dist_obs_out = dev_dist_obs;
  return MC_OK;
}

int mc_set_minimap_obs(void* env, double* dev_minimap_obs) {
  Env* E = as_env(env);
  if (!E || !dev_minimap_obs) return fail(MC_EINVAL, "mc_set_minimap_obs: null argument");
  if (E->cfg.mini_map_rad <= 0) return fail(MC_EINVAL, "mc_set_minimap_obs: config has mini_map_rad = 0");
  E->mini_obs = dev_minimap_obs;
  return MC_OK;
}

// Diagnostic builds only: point the kernels at a [B][16] u64 stamp buffer.
int mc_debug_stamps(void* env, uint64_t* dev_stamps) {
  Env* E = as_env(env);
  if (!E) return fail(MC_EINVAL, "mc_debug_stamps: null env");
#if defined(MC_STAMPS) || defined(MC_DIST_STAMPS)
  E->s.stamps = dev_stamps;
  return MC_OK;
#else
  (void)dev_stamps;
  return fail(MC_EINVAL, "not a -DMC_STAMPS build");
#endif
}

int mc_check(void* env, void* stream) {
  Env* E = as_env(env);
  if (!E) return fail(MC_EINVAL, "mc_check: null env");
  hipStream_t st = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(E->device));
  uint32_t err = 0;
  HIP_TRY(hipMemcpyAsync(&err, E->s.err, 4, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (err) {
    HIP_TRY(hipMemsetAsync(E->s.err, 0, 4, st));
    HIP_TRY(hipStreamSynchronize(st));
    return fail(MC_EDEVICE, "device error word 0x%x (1=window 4=placement 8=inject)", err);
  }
  return MC_OK;
}

}  // extern "C"
