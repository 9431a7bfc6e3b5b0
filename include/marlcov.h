/*
 * marlcov.h — C ABI of libmarlcov.so, the MI355X (gfx950) batched coverage
 * environment.  This is the drop-in boundary for the reference's env hot path
 * (ExistentialRobotics/MARL-Coverage, Environments/dec_grid_rl.py:DecGridRL).
 *
 * The reference has no FFI: its boundary is the duck-typed Python class
 * DecGridRL (dec_grid_rl.py:21).  Each entry point below replaces one piece of
 * that class for a whole batch of environments at once; the Python facade
 * (marl-coverage_amd/dec_grid_rl.py) and the batched env (batch_env.py) bind
 * them with ctypes.
 *
 * Conventions
 *   - Plain C types only.  `stream` is a hipStream_t passed as void* (NULL =
 *     the null stream).  Every `dev_*` pointer is HIP device memory owned by
 *     the caller; env state is owned by the library.
 *   - Every call returns 0 on success and a negative MC_E* code on error; the
 *     message is in mc_last_error() (thread-local).  Nothing throws across
 *     the ABI.  Work is stream-ordered and asynchronous unless noted.
 *   - One handle per (device, stream); a handle is not thread-safe.
 *   - Coordinates are in the PADDED grid (the reference pads every map with a
 *     -1 border, dec_grid_rl.py:471-472): x in [0, width), y in [0, length).
 *   - Bit maps (MC_FIELD_FREE/OBST/VISITED/GRID_*) are 8x8-cell tiles, bit
 *     8*r + c of tile (ti, tj) = cell (8*ti + r, 8*tj + c), grouped 4x4 into
 *     128-byte blocks: uint64 [...][tile_rows/4][tile_cols/4][4][4], tile
 *     (ti, tj) at block (ti/4, tj/4), slot (ti%4, tj%4).  Cells beyond the
 *     grid (edge and padding tiles) are set in GRID_NEG (out of bounds =
 *     blocked) and clear in every other map.
 */
#ifndef MARLCOV_H
#define MARLCOV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MARLCOV_ABI_VERSION 9

enum {
  MC_OK = 0,
  MC_EINVAL = -1,   /* bad argument / unsupported config                    */
  MC_EHIP = -2,     /* HIP runtime error                                     */
  MC_ESTATE = -3,   /* call out of order (e.g. step before grids)            */
  MC_EDEVICE = -4   /* a kernel raised its device error word (mc_check)      */
};

enum { MC_SENSOR_LIDAR = 0, MC_SENSOR_SQUARE = 1 };

/* action byte meanings (per agent), dec_grid_rl.py:131-145 */
enum {
  MC_ACT_RIGHT = 0,      /* x + 1 */
  MC_ACT_UP = 1,         /* y + 1 */
  MC_ACT_LEFT = 2,       /* x - 1 */
  MC_ACT_DOWN = 3,       /* y - 1 */
  /* 4..254: no-op, no penalty (any non-{0,1,2,3} value in the reference)   */
  MC_ACT_SENTINEL = 255  /* in agent 0's byte: the whole env step is the
                            reference's `action == None or -1` path
                            (dec_grid_rl.py:104-107): done=1, reward=0, no
                            state change, observations still written        */
};

/* Environment configuration: the reference env_config keys
 * (dec_grid_rl.py:49-75, lidar.py:8-9, squaresensor.py:12) plus batch extras. */
typedef struct mc_config {
  int32_t num_envs;           /* B (batch extra)                              */
  int32_t num_agents;         /* 'numrobot', 1..64                            */
  int32_t width;              /* padded grid rows    (unpadded W + 2)         */
  int32_t length;             /* padded grid columns (unpadded L + 2)         */
  int32_t num_grids;          /* G grids in the device pool (>= 1)            */
  int32_t sensor_type;        /* MC_SENSOR_*   ('sensor_type')                */
  int32_t num_beams;          /* lidar 'num_lasers' (any count >= 1)          */
  int32_t square_radius;      /* square_sensor 'range'                        */
  double lidar_range;         /* lidar 'range' (float64 compare, lidar.py:52) */
  int32_t egoradius;          /* 'egoradius'                                  */
  int32_t pad;                /* max(egoradius, mini_map_rad) (:78)           */
  double collision_penalty;   /* 'collision_penalty'                          */
  double terminal_reward;     /* 'terminal_reward'                            */
  double done_thresh;         /* 'done_thresh' (initial, per env)             */
  double done_incr;           /* 'done_incr'                                  */
  int32_t maxsteps;           /* 'maxsteps' (done when currstep == maxsteps)  */
  int32_t comm_radius;        /* 'comm_radius' (Chebyshev)                    */
  int32_t map_sharing;        /* 'map_sharing'                                */
  int32_t single_square_tool; /* 'single_square_tool'                         */
  int32_t dist_reward;        /* 'dist_reward' (float obs layer: mc_set_dist_obs) */
  int32_t dijkstra_input;     /* 'dijkstra_input'                             */
  int32_t auto_reset;         /* batch extra: re-place agents on done         */
  int32_t reset_grid_mode;    /* 0: keep the env's grid on reset;
                                 1: draw a grid uniformly from the pool       */
  int32_t mini_map_rad;       /* 'mini_map_rad' (> 0: float64 minimap layers
                                 3-4 via mc_set_minimap_obs; pad >= it)       */
  uint64_t seed;              /* batch extra: device Philox seed              */
  /* Global ids (batch extras): env e of this handle is global env
   * env_offset + e and pool grid g is global grid grid_offset + g.  Every
   * device random stream (start-cell draws, the grid pick, mc_generate_grids,
   * mc_random_actions) is keyed by the global id, so a shard of a global batch
   * reproduces those envs bit for bit whatever the number of GPUs.          */
  uint32_t env_offset;
  uint32_t grid_offset;
} mc_config;

/* Derived geometry (mc_query). */
typedef struct mc_layout {
  int32_t tile_rows;          /* ceil(width / 8) rounded up to a multiple of 4  */
  int32_t tile_cols;          /* ceil(length / 8) rounded up to a multiple of 4 */
  int32_t window_half;        /* H = max(ceil(range), egoradius)              */
  int32_t window_tiles;       /* TW: tiles per side staged per agent          */
  int32_t obs_layers;         /* Lc ((mini_map_rad > 0 ? 5 : 3) + dist_reward
                                 + dijkstra_input, dec_grid_rl.py:322-332)    */
  int32_t obs_side;           /* E = 2*egoradius + 1                          */
  int64_t obs_bytes_per_env;  /* N*Lc*E*E (uint8 obs)                         */
  int64_t mask_words_per_agent; /* tile_rows * tile_cols (one map)            */
  int64_t state_bytes;        /* device bytes owned by the handle             */
} mc_layout;

/* State fields for mc_get_state / mc_set_state (device-to-device copies).  */
enum {
  MC_FIELD_POS = 0,          /* int32 [B][N][2] (x, y)                         */
  MC_FIELD_MOVED = 1,        /* uint64 [B]  bit i: robot i is in robot_pad     */
  MC_FIELD_FREE = 2,         /* uint64 [B][N][map] _free_pad (map: see above)  */
  MC_FIELD_OBST = 3,         /* uint64 [B][N][map] _obst_pad                   */
  MC_FIELD_VISITED = 4,      /* uint64 [B][map]    _visited                    */
  MC_FIELD_FREE_COUNT = 5,   /* uint32 [B]  count_nonzero(_free_pad > 0)       */
  MC_FIELD_VISITED_COUNT = 6,/* uint32 [B]  sum(_visited)                      */
  MC_FIELD_CURRSTEP = 7,     /* int32  [B]  _currstep                          */
  MC_FIELD_DONE_THRESH = 8,  /* double [B]  _done_thresh                       */
  MC_FIELD_ENV_GRID = 9,     /* int32  [B]  grid pool index of each env        */
  MC_FIELD_EPISODE = 10,     /* uint32 [B]  resets so far (RNG counter)        */
  MC_FIELD_NUMFREE = 11,     /* int32  [G]  count_nonzero(grid > 0) per grid   */
  MC_FIELD_GRID_NEG = 12,    /* uint64 [G][map] grid < 0                       */
  MC_FIELD_GRID_POS = 13,    /* uint64 [G][map] grid > 0                       */
  /* dist_reward configs only (MC_EINVAL otherwise):                           */
  MC_FIELD_DIST_MW = 14,     /* int32 [B][N][2] (M, witness): M = max of the map's
                                L1 distance transform (-1 = unknown: the next
                                POST runs the full transform), witness = a cell
                                with d == M, (x << 16) | (y & 0xFFFF), map coords */
  MC_FIELD_DIST_LISTED = 15, /* int32 [1] maps the last POST sent to the full
                                transform (read-only diagnostic)               */
  /* episode record (read-only), written when an env reports done, before an
     auto-reset clears the counters: the Utils/utils.py:141 statistic       */
  MC_FIELD_EP_PC = 16,       /* double [B] percent_covered() at the episode end */
  MC_FIELD_EP_LEN = 17,      /* int32  [B] _currstep at the episode end        */
  /* dijkstra_input configs only (MC_EINVAL otherwise):                        */
  MC_FIELD_DJ_LISTED = 18,   /* int32 [1] (env, agent) paths the last step sent
                                to the full-map BFS: nearest unexplored cell
                                more than 24 steps away (read-only diagnostic) */
  /* dist_reward configs only:                                                 */
  MC_FIELD_DIST_CACHED = 19, /* int32 [1] of the maps the last POST listed, those
                                the top-cell cache served without a full
                                transform (read-only diagnostic)               */
  MC_FIELD_DIST_TOTALS = 20, /* uint64 [4] cumulative since mc_create: maps the
                                POSTs listed, of them served by the top-cell
                                cache, fully transformed, and POST launches
                                (read-only diagnostic: a caller takes deltas;
                                the bench's C5 design bytes)    */
  MC_FIELD_COUNT = 21
};

int32_t mc_abi_version(void);
const char* mc_last_error(void);
/* sizeof(mc_config) (which=0) / sizeof(mc_layout) (1) / sizeof(mc_sg_config)
 * (2) / sizeof(mc_sg_layout) (3): lets an FFI binding verify its struct
 * mirrors. */
int64_t mc_struct_size(int32_t which);

/* Build-time constants a caller prices or sizes work with (ABI v9): the
 * top-cell cache's cells per map (kDistK, MC_DIST_K build knob), its
 * threshold (kDistT: the cache holds every cell with d >= M0 - kDistT) and
 * the largest extended grid (rows) the distance transform takes.  -1 for an
 * unknown `which`. */
enum { MC_PARAM_DIST_CACHE_CELLS = 0, MC_PARAM_DIST_T = 1, MC_PARAM_DIST_MAX_ROWS = 2 };
int64_t mc_build_param(int32_t which);

/* Allocate device state for cfg->num_envs envs on HIP device `hip_device`.
 * Replaces DecGridRL.__init__ (dec_grid_rl.py:30-89) minus the first reset. */
int mc_create(const mc_config* cfg, int hip_device, void** out_env);
void mc_destroy(void* env);
int mc_query(void* env, mc_layout* out);

/* Lidar beam table, host memory [num_beams][3] float64 (xinc, yinc, distinc),
 * computed by the caller exactly as lidar.py:38-48 does (per-theta NumPy
 * scalar cos/sin, normalise by max(|.|), sqrt).  Synchronous upload. */
int mc_set_beam_table(void* env, const double* host_table, int32_t num_beams);

/* Upload the grid pool: dev_grids int8 [num_grids][width][length], values
 * <0 obstacle, 0 traversable-but-not-free, >0 free; the caller has already
 * added the -1 border.  Replaces the np.pad in reset (dec_grid_rl.py:471). */
int mc_set_grids(void* env, const int8_t* dev_grids, int32_t num_grids, void* stream);

/* Synthetic pool: grid g interior cells are obstacles with probability
 * p_obst (Philox(seed, grid_offset + g)), border -1.  Same distribution as gridgen
 * (Utils/gridmaker.py:127-128); not the same bits. */
int mc_generate_grids(void* env, uint64_t seed, double p_obst, void* stream);

/* Synthetic per-agent action bytes for step `step`: dev_actions uint8 [B][N]
 * uniform in {0..3} from Philox(seed, global env id, step) (SURVEY 8(d)
 * "Actions (GPU)"), so a shard draws exactly the actions its envs draw in one
 * big batch. */
int mc_random_actions(void* env, uint64_t seed, int32_t step, uint8_t* dev_actions, void* stream);

/* Name of the env-kernel instantiation the next mc_step / mc_reset launches
 * (compiled shape or the generic kernel, lanes per workgroup, envs per
 * workgroup), e.g. "env_kernel<64,2,u32,C2>", followed by " +fan(S/P)" when
 * a dense lidar set marches by sectors (S sectors, P special beams) instead
 * of by rays.  Diagnostic: lets tests show which specialisation they cover.
 * The string stays valid until the calling thread's next call. */
const char* mc_kernel_variant(void* env);

/* Which pool grid each env uses (int32 [B], device). */
int mc_set_env_grids(void* env, const int32_t* dev_env_grid, void* stream);

/* Reset (dec_grid_rl.py:449-531) the envs with dev_env_mask[e] != 0 (NULL =
 * all).  dev_pos int32 [B][N][2] injects start cells (NULL = device Philox
 * rejection draw, same acceptance rule as :491-502).  Writes uint8 obs
 * [B][N][Lc][E][E] for every env (non-reset envs: current-state obs) and,
 * when dev_adj != NULL, the comm graph uint8 [B][N][N] (:374-391). */
int mc_reset(void* env, const uint8_t* dev_env_mask, const int32_t* dev_pos,
             void* dev_obs, uint8_t* dev_adj, void* stream);

/* One step of every env (dec_grid_rl.py:91-169) with per-agent action bytes
 * dev_actions uint8 [B][N] (MC_ACT_*).  Writes reward float64 [B], done uint8
 * [B], obs uint8 [B][N][Lc][E][E] and optionally the comm graph [B][N][N].
 * With cfg.auto_reset, an env that reports done (the sentinel step included)
 * is reset in the same launch and its obs are the first obs of the new
 * episode; MC_FIELD_EP_PC / EP_LEN keep the finished episode's record. */
int mc_step(void* env, const uint8_t* dev_actions, double* dev_reward,
            uint8_t* dev_done, void* dev_obs, uint8_t* dev_adj, void* stream);

/* num_steps consecutive mc_step calls in one call: step k reads the action
 * bytes at dev_actions + k * actions_stride and writes reward / done / obs /
 * adjacency at their pointer + k * stride (byte strides; 0 = every step
 * overwrites the same buffer; dev_adj may be NULL).  Each step is launched
 * exactly as mc_step launches it (one env-kernel launch, plus the dist /
 * dijkstra launches of the config), stream-ordered.  For callers whose
 * actions are known ahead (open-loop rollouts, benchmarks): one FFI crossing
 * instead of num_steps.  Same semantics as the reference's step
 * (dec_grid_rl.py:91-169) applied num_steps times.  Strides are in bytes
 * (0: every step writes the same buffer); reward_stride must be a multiple of
 * 8.  Arguments are checked before anything is enqueued; if a launch of step
 * k fails, steps 0..k-1 are already enqueued (the env has advanced k steps)
 * and mc_last_error() names k. */
int mc_step_many(void* env, const uint8_t* dev_actions, int64_t actions_stride, int32_t num_steps,
                 double* dev_reward, int64_t reward_stride, uint8_t* dev_done, int64_t done_stride,
                 void* dev_obs, int64_t obs_stride, uint8_t* dev_adj, int64_t adj_stride,
                 void* stream);

/* Device-to-device copy of a state field into / out of caller memory.
 * `bytes` must equal the field size (mc_field_bytes). */
int64_t mc_field_bytes(void* env, int32_t field);
int mc_get_state(void* env, int32_t field, void* dev_dst, int64_t bytes, void* stream);
int mc_set_state(void* env, int32_t field, const void* dev_src, int64_t bytes, void* stream);

/* dist_reward (dec_grid_rl.py:222-223,239-240,260-282,350-352): register the
 * caller's float32 [B][N][E][E] buffer that every mc_reset / mc_step fills
 * with the distance-map crop (obs layer 3; the uint8 obs hold 0 there).
 * Required before the first reset when cfg.dist_reward != 0.  With
 * dijkstra_input as well, layer 3 of the uint8 obs is the dijkstra path and
 * layer 4 is 0, as in the reference (the dist crop is overwritten, :354). */
int mc_set_dist_obs(void* env, float* dev_dist_obs);

/* mini_map_rad > 0 (dec_grid_rl.py:360-370): register the caller's float64
 * [B][N][2][E][E] buffer that every mc_reset / mc_step fills with obs layers 3
 * and 4, cv2.resize(INTER_LINEAR) of the agent's free / obstacle maps cropped
 * with radius mini_map_rad (OpenCV's generic CV_64F path; parity vs OpenCV
 * unpinned).  The uint8 obs hold 0 in layers 3.. (the minimap overwrites the
 * dist / dijkstra layer in the reference).  Required before the first reset. */
int mc_set_minimap_obs(void* env, double* dev_minimap_obs);

/* Synchronise `stream` and report (then clear) the device error word. */
int mc_check(void* env, void* stream);

/* ==========================================================================
 * SuperGridRL — the centralized, fully observed env variant
 * (Environments/super_grid_rl.py:18-463).  A separate
 * handle type with the same conventions as above, except that grids are NOT
 * padded (SuperGridRL never pads, :357-366) and maps are row bitboards:
 * uint64 [W][ceil(L/64)], bit (y & 63) of word (x, y >> 6) = cell (x, y).
 *
 * The state the reference returns from every reset/step (get_state,
 * :305-317: P position layers, observed obstacles, _free, distance map) lives
 * in two caller buffers registered with mc_sg_set_obs and MAINTAINED by the
 * library: reset rewrites them whole, a step updates only the cells it
 * changes (robot cells, sensed windows) and rewrites the distance layer.  The
 * caller reads them and must not write them.
 * ======================================================================== */

typedef struct mc_sg_config {
  int32_t num_envs;           /* B (batch extra)                              */
  int32_t num_agents;         /* 'numrobot', 1..64                            */
  int32_t width;              /* grid rows W (unpadded)                       */
  int32_t length;             /* grid columns L (unpadded)                    */
  int32_t num_grids;          /* G grids in the device pool (>= 1)            */
  int32_t senseradius;        /* 'senseradius', 0..15                         */
  double collision_penalty;   /* 'collision_penalty'                          */
  double free_penalty;        /* 'free_penalty'                               */
  double terminal_reward;     /* 'terminal_reward'                            */
  double done_thresh;         /* 'done_thresh' (initial, per env)             */
  double done_incr;           /* 'done_incr'                                  */
  int32_t dist_reward;        /* 'dist_reward'                                */
  int32_t use_scanning;       /* 'use_scanning' (one position layer)          */
  int32_t maxsteps;           /* batch extra: done when currstep == maxsteps
                                 (the episode cut of Utils/utils.py:25-28);
                                 0 = never, as in SuperGridRL.done()         */
  int32_t auto_reset;         /* batch extra: reset an env that reports done  */
  int32_t reset_grid_mode;    /* 0: keep the env's grid; 1: draw from the pool */
  int32_t pad_;
  uint64_t seed;              /* batch extra: device Philox seed              */
  uint32_t env_offset;        /* global id of env 0 (see mc_config)           */
  uint32_t grid_offset;       /* global id of pool grid 0                     */
} mc_sg_config;

typedef struct mc_sg_layout {
  int32_t pos_layers;         /* P: N, or 1 with use_scanning (:330-341)      */
  int32_t obs_layers;         /* P + 2 uint8 layers (positions, obstacles, free) */
  int32_t row_words;          /* ceil(L / 64)                                 */
  int32_t pad_;
  int64_t state_bytes;        /* device bytes owned by the handle             */
} mc_sg_layout;

enum {
  MC_SG_FIELD_POS = 0,        /* int32  [B][N][2] (_xinds, _yinds)            */
  MC_SG_FIELD_COVERED = 1,    /* uint64 [B][W][RW] _free == 0 (sensed)        */
  MC_SG_FIELD_OBST = 2,       /* uint64 [B][W][RW] _observed_obstacles        */
  MC_SG_FIELD_COV_COUNT = 3,  /* uint32 [B] count_nonzero(_free < 1)          */
  MC_SG_FIELD_CURRSTEP = 4,   /* int32  [B] _currstep                         */
  MC_SG_FIELD_DONE_THRESH = 5,/* double [B] _done_thresh                      */
  MC_SG_FIELD_A_PREV = 6,     /* int32  [B] a_prev (-1 = None)                */
  MC_SG_FIELD_ENV_GRID = 7,   /* int32  [B] grid pool index                   */
  MC_SG_FIELD_EPISODE = 8,    /* uint32 [B] resets so far (RNG counter)       */
  MC_SG_FIELD_NUMPOS = 9,     /* int32  [G] count_nonzero(grid > 0)           */
  MC_SG_FIELD_GRID_NEG = 10,  /* uint64 [G][W][RW] grid < 0                   */
  MC_SG_FIELD_GRID_POS = 11,  /* uint64 [G][W][RW] grid > 0                   */
  MC_SG_FIELD_EP_PC = 12,     /* double [B] percent_covered() at the last done (read-only) */
  MC_SG_FIELD_EP_LEN = 13,    /* int32  [B] _currstep at the last done (read-only) */
  MC_SG_FIELD_COUNT = 14
};

/* Replaces SuperGridRL.__init__ (:27-72) minus the first reset. */
int mc_sg_create(const mc_sg_config* cfg, int hip_device, void** out_env);
void mc_sg_destroy(void* env);
int mc_sg_query(void* env, mc_sg_layout* out);
/* dev_grids int8 [num_grids][W][L], values < 0 obstacle, 0, > 0 free. */
int mc_sg_set_grids(void* env, const int8_t* dev_grids, int32_t num_grids, void* stream);
/* Bernoulli pool: every cell an obstacle with probability p_obst (gridgen's
 * distribution, Utils/gridmaker.py:127-128; not its bits). */
int mc_sg_generate_grids(void* env, uint64_t seed, double p_obst, void* stream);
int mc_sg_set_env_grids(void* env, const int32_t* dev_env_grid, void* stream);
/* Register the state buffers (see above): dev_planes uint8 [B][P+2][W][L]
 * (layers 0..P-1 robot positions, P observed obstacles, P+1 _free),
 * dev_dist float32 [B][W][L] (get_distance_map, :281-303).  Required before
 * the first reset. */
int mc_sg_set_obs(void* env, uint8_t* dev_planes, float* dev_dist);
/* SuperGridRL.reset (:343-399) of the envs with dev_env_mask[e] != 0 (NULL =
 * all): start cells injected (dev_pos int32 [B][N][2]) or drawn on the device
 * (Philox rejection, the acceptance rule of :378-388); _done_thresh and
 * a_prev are kept, as in the reference. */
int mc_sg_reset(void* env, const uint8_t* dev_env_mask, const int32_t* dev_pos, void* stream);
/* SuperGridRL.step (:74-225) of every env.  dev_actions uint8 [B][N]: the
 * base-4 digits of the joint action, slot 0 first (:93-98); 0 = x-1, 1 = x+1,
 * 2 = y+1, 3 = y-1 (:131-174); 4..254 no-op; 255 in slot 0 = the sentinel
 * path (:88-90: reward 0, done, no state change).  dev_quot int32 [B]
 * (nullable = all 0): action // 4**N, the value motion_penalty sees (:203-208);
 * >= 4 raises the device error (the reference's KeyError).  Writes reward
 * float64 [B] and done uint8 [B], and updates the registered state buffers. */
int mc_sg_step(void* env, const uint8_t* dev_actions, const int32_t* dev_quot, double* dev_reward,
               uint8_t* dev_done, void* stream);
int64_t mc_sg_field_bytes(void* env, int32_t field);
int mc_sg_get_state(void* env, int32_t field, void* dev_dst, int64_t bytes, void* stream);
/* Uploads mark the state buffers for a full rewrite at the next call. */
int mc_sg_set_state(void* env, int32_t field, const void* dev_src, int64_t bytes, void* stream);
/* Synchronise and report (then clear) the device error word:
 * 4 = placement failed, 8 = bad injected cell, 16 = motion_penalty KeyError. */
int mc_sg_check(void* env, void* stream);

/* Diagnostics: in a -DMC_STAMPS build, record per-phase s_memtime stamps of
 * every env into dev_stamps uint64 [B][16]; MC_EINVAL in normal builds. */
int mc_debug_stamps(void* env, uint64_t* dev_stamps);

#ifdef __cplusplus
}
#endif
#endif /* MARLCOV_H */
