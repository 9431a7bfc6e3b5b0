"""Throughput benchmark of the batched coverage env step (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c4|c5] [--envs B]

One "step" = one launch of the HIP env kernel advancing every env of this
GPU's shard by one timestep (all agents move, sense, merge, reward, done,
obs, auto-reset).  Inputs (grids, state, per-step action bytes) are resident
in HBM before the timed region.  N>1: one process per GPU, each rank owns an
independent env shard (weak scaling, no collective on the step path); RCCL
is used once after timing for the scalar episode-return all-reduce and the
max-over-ranks time.  Under torchrun the ranks come from its env; a plain
`python bench.py --gpus N` starts `torch.distributed.run --nproc-per-node N`
itself as a child (launch_ranks) and exits with its code.  A world size that
differs from --gpus, or more RCCL ranks than visible GPUs, exits non-zero.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node), 4-agent 128×128 grid, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

BASE = dict(maxsteps=1000, collision_penalty=5, done_thresh=1, done_incr=0, terminal_reward=30,
            dist_reward=0, train_maxsteps=1000, test_maxsteps=1000, egoradius=2, mini_map_rad=0,
            comm_radius=0, allow_comm=0, map_sharing=0, single_square_tool=0, dijkstra_input=0,
            sensor_type="lidar")

# SURVEY.md §8(d) workloads (configs[1] = C2 is the metric's N=1 workload)
CONFIGS = {
    "c2": dict(numrobot=4, width=128, sensor_config={"num_lasers": 21, "range": 10}, envs=4096,
               desc="C2: 4 agents, 128x128 grid p_obst=0.1, lidar 21 beams R=10, egoradius 2"),
    "c4": dict(numrobot=8, width=256, sensor_config={"num_lasers": 360, "range": 20}, envs=8192,
               desc="C4: 8 agents, 256x256 grid p_obst=0.1, lidar 360 beams R=20, egoradius 2"),
    "c5": dict(numrobot=16, width=512, sensor_config={"num_lasers": 21, "range": 10}, envs=8192,
               extra={"dist_reward": 1}, maxsteps=2000,
               desc="C5: 16 agents, 512x512 grid p_obst=0.1, lidar 21 beams R=10, dist_reward "
                    "(frontier-coverage reward, float32 distance layer)"),
    # C2 with the dijkstra_input obs layer (BSA/BA*-style
    # controllers); not a BASELINE metric config
    "c2_dijkstra": dict(numrobot=4, width=128, sensor_config={"num_lasers": 21, "range": 10}, envs=4096,
                        extra={"dijkstra_input": 1},
                        desc="C2 + dijkstra_input obs layer (4 layers)"),
    # the centralized SuperGridRL on C2's shape (full-map
    # state every step: P+2 uint8 layers + float32 distance layer); not a
    # BASELINE metric config
    "sg_c2": dict(env="super", numrobot=4, width=128, envs=4096, sensor_config={"range": 0},
                  sg=dict(senseradius=2, free_penalty=0.2, dist_reward=1, use_scanning=0),
                  desc="SuperGridRL: 4 agents, 128x128 grid p_obst=0.1, senseradius 2, free_penalty 0.2, "
                       "dist_reward, full-map state (4 position + obstacle + free uint8 layers, "
                       "float32 distance layer), episode cut 1000"),
}

SG_BASE = dict(train_maxsteps=1000, test_maxsteps=1000, collision_penalty=5, done_thresh=1, done_incr=0,
               terminal_reward=30)


def sg_algorithmic_bytes_per_env_step(n_agents, r, W, L):
    """SuperGridRL: per env the float32 distance layer write
    (4 B per cell) and the read of the covered bit map its transform needs
    (W * ceil(L/64) * 8 B); per agent the window bits of grid / covered /
    obstacle read (3 * ceil(s^2/8)), covered / obstacle ORs (2 * ceil(s^2/8)),
    the obstacle / free layer bytes of the window (2 * s^2), two position-layer
    bytes, 1 B action and 8 B position r/w (s = 2r+1); per env 32 B."""
    s2 = (2 * r + 1) ** 2
    bits = math.ceil(s2 / 8)
    return W * L * 4 + W * math.ceil(L / 64) * 8 + n_agents * (5 * bits + 2 * s2 + 2 + 1 + 8) + 32


def algorithmic_bytes_per_env_step(n_agents, beam_range, ego, layers=3, full_map_cells=0):
    """per agent s^2 (int8 grid window) + 4*ceil(s^2/8) (free and
    obst bit windows, read+write) + 2*ceil(s^2/8) (union window read+write) +
    obs bytes + 1 (action) + 8 (position r/w); per env 32 B.  Map-wide layers
    add a read of the agent's free and obst bit maps over `full_map_cells`
    cells: 2*ceil(cells/8) per agent -- C5's distance map over the whole map,
    as §8(d) prices it; dijkstra_input over the 64 x 64 BFS window its kernel
    reads (the paths it lists for the full map are extra)."""
    s = 2 * math.ceil(beam_range) + 1
    bits = math.ceil(s * s / 8)
    obs = layers * (2 * ego + 1) ** 2
    full = 2 * math.ceil(full_map_cells / 8) if full_map_cells else 0
    return n_agents * (s * s + 6 * bits + obs + 1 + 8 + full) + 32


DJ_WINDOW_CELLS = 64 * 64  # csrc/mc_dijkstra.hip: dijkstra_window_kernel

def dist_cache_bytes():
    """Bytes of one map's top-cell cache: kDistK (the library's build
    constant, mc_build_param) x (i32 cell + i32 d) + the 32-B header."""
    from marlcov import _lib
    return _lib.load().mc_build_param(_lib.PARAM_DIST_CACHE_CELLS) * 8 + 32


def c5_design_bytes_per_step(B, n_agents, beam_range, ego, ext_side, listed, served, full, launches):
    """C5 (dist_reward) design algorithmic bytes of one step of B envs
    (DESIGN.md §5): every env-step's windowed SURVEY 8(d) part (the 8(d)
    formula without its full-map term: 15,408 B per env at C5); plus, per
    step, the maps that really ran a full distance transform (one read of the
    map's free bit map, ceil(ext_side^2 / 8) B, and the write of its top-cell
    cache), the maps the cache served (one read of their cache), and one
    4-B list entry per listed map.  listed / served / full are the
    MC_FIELD_DIST_TOTALS deltas over `launches` POST launches.  SURVEY 8(d)'s
    C5 figure prices a full-map read of every agent's map every step
    (1,088,720 B per env-step); the witness test and the top-cell cache skip
    most of those reads, so that figure is an upper-bound price, not the work
    timed."""
    window = algorithmic_bytes_per_env_step(n_agents, beam_range, ego, layers=3 + 4)
    per_map = math.ceil(ext_side * ext_side / 8)
    cb = dist_cache_bytes()
    extra = full * (per_map + cb) + served * cb + listed * 4
    return B * window + (extra / launches if launches else 0.0)


# ---------------------------------------------------------------------------
# CPU baseline: the oracle (NumPy restatement of the reference step, keeping its
# per-cell Python beam march and full-map copies) in P independent processes.
# Runs BEFORE the GPU is touched (fork-safe).
# ---------------------------------------------------------------------------
# at least 2 s per process, and at C4 / C5 at least 20 steps
CPU_MIN_STEPS = {"c4": 20, "c5": 20}


def _cpu_worker(args):
    seed, secs, cfgname = args
    min_steps = CPU_MIN_STEPS.get(cfgname, 8)
    import numpy as np
    from oracle.cpu_ref import DecGridRLRef

    c = CONFIGS[cfgname]
    if c.get("env") == "super":
        return _cpu_worker_super(seed, secs, c)
    cfg = dict(BASE, numrobot=c["numrobot"], sensor_config=c["sensor_config"],
               allow_even_beams=True, **c.get("extra", {}))
    rs = np.random.RandomState(1000 + seed)
    grid = rs.choice([1.0, -1.0], size=(c["width"], c["width"]), p=[0.9, 0.1])
    np.random.seed(seed)
    env = DecGridRLRef([grid], cfg)
    acts = rs.randint(0, 4, size=(4096, c["numrobot"]))
    n = 0
    t0 = time.perf_counter()
    while True:
        _, _, done = env.step(acts[n % 4096])
        n += 1
        if done:
            env.reset(False, None)
        if n >= min_steps and n % 8 == 0 and time.perf_counter() - t0 >= secs:
            break
    return n, time.perf_counter() - t0


def _cpu_worker_super(seed, secs, c):
    import numpy as np
    from oracle.super_ref import SuperGridRLRef

    cfg = dict(SG_BASE, numrobot=c["numrobot"], **c["sg"])
    rs = np.random.RandomState(1000 + seed)
    grid = rs.choice([1.0, -1.0], size=(c["width"], c["width"]), p=[0.9, 0.1])
    np.random.seed(seed)
    env = SuperGridRLRef([grid], cfg)
    N = c["numrobot"]
    acts = rs.randint(0, 4 ** N, size=4096)
    n = 0
    t0 = time.perf_counter()
    while True:
        _, _, done = env.step(int(acts[n % 4096]))
        n += 1
        if done or env._currstep == cfg["train_maxsteps"]:  # the episode cut of Utils/utils.py:25-28
            env.reset(False, None)
        if n % 8 == 0 and time.perf_counter() - t0 >= secs:
            break
    return n, time.perf_counter() - t0


def cpu_baseline(cfgname, procs, secs):
    import multiprocessing as mp

    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(i, secs, cfgname) for i in range(procs)])
    rate = sum(n / t for n, t in res)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    port = ("oracle/super_ref.py (SuperGridRL step restated, per-cell Python sense loop kept)"
            if CONFIGS[cfgname].get("env") == "super" else
            "oracle/cpu_ref.py (reference step restated, per-cell Python beam march kept)")
    out = {"value": round(rate, 2), "unit": "env-steps/s", "cores": procs, "kind": "port",
           "sample": f"{procs} processes x {secs:.1f} s, one env each, {CONFIGS[cfgname]['desc']}, "
                     f"random joint actions; {port}; host CPU: {cpu}"}
    ratio = port_over_reference(cfgname)
    if ratio:  # the port's rate over the reference's own step, same core (build container)
        out["port_over_reference"] = ratio
        out["reference_equiv_value"] = round(rate / ratio, 2)
        out["calibration"] = CALIBRATION
    return out


CALIBRATION = "profiles/r4/cpu_calibration.json"


def port_over_reference(cfgname):
    """tools/calibrate_cpu.py: the oracle's single-core rate over the imported
    reference DecGridRL.step's on one core of the build container, same grid,
    actions and seeds (the reference cannot travel to the GPU box)."""
    try:
        with open(os.path.join(ROOT, CALIBRATION)) as f:
            return json.load(f)["results"][cfgname]["port_over_reference"]
    except (OSError, ValueError, KeyError):
        return None


def load_traffic(cfgname, full=False):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (if any);
    full=True: the whole record (bytes, the profiled step time and phase)."""
    path = os.path.join(ROOT, "profiles", f"traffic_{cfgname}.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    return rec if full else rec.get("hbm_bytes_per_launch")


def measured_traffic(cfgname, warmup, steps):
    """The HBM bytes a timed step really moves (PMC passes, profiles/
    traffic_<config>.json) over the step time of the SAME profiled run (same
    build, same episode phase), with the phase it was taken in; `matches`
    says whether this bench run times the same phase."""
    rec = load_traffic(cfgname, full=True)
    if not rec or not rec.get("hbm_bytes_per_launch") or not rec.get("step_mean_us"):
        return None
    b, us = rec["hbm_bytes_per_launch"], rec["step_mean_us"]
    w, k = rec.get("warmup"), rec.get("steps")
    return {"bytes_per_step": b, "step_us": us, "achieved": round(b / (us * 1e-6) / 1e9, 2),
            "frac": round(b / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 5),
            "phase": f"steps {w + 1}..{w + k} after the first reset" if w is not None and k else "unrecorded",
            "matches_this_run": w == warmup if w is not None else None,
            "from": f"profiles/traffic_{cfgname}.json (FETCH_SIZE x2 + WRITE_SIZE per timed step, "
                    "rocprofv3 kernel means of the same run)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (default: config's)")
    ap.add_argument("--global-envs", type=int, default=None,
                    help="split this fixed global batch over the ranks (strong scaling, shard_range) "
                         "instead of --envs per GPU (weak scaling)")
    # the GPU box's host share is 16 CPUs per GPU (os.cpu_count() there shows
    # the whole machine): one single-env oracle process per core
    ap.add_argument("--cpu-procs", type=int, default=16)
    ap.add_argument("--cpu-secs", type=float, default=2.5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--maxsteps", type=int, default=None,
                    help="episode length (auto-reset on done); default: the config's (1000, C5 2000)")
    ap.add_argument("--launch", default="native", choices=["native", "stream", "graph", "events"],
                    help="native: the K launches issued by one C-ABI call (mc_step_many, one kernel "
                         "launch per step); stream: K back-to-back Python/ctypes mc_step calls; graph: "
                         "uploaded hipGraph replay; events: per-launch HIP events")
    ap.add_argument("--eager", action="store_true", help="alias of --launch events")
    ap.add_argument("--events", default="around", choices=["around", "after-first", "none"],
                    help="native launch: where the HIP events that time the kernels sit in the timed region. "
                         "around: before the first launch and after the last (kernel_us over K); after-first: "
                         "after the first launch (a separate 1-launch mc_step_many call) and after the last "
                         "(kernel_us over K - 1, no marker packet ahead of the first kernel); none: no events "
                         "(kernel_us null)")
    ap.add_argument("--sync", default="default", choices=["default", "spin"],
                    help="spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before the device is initialised, so "
                         "the host synchronize that closes the timed region spin-waits instead of sleeping")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group for N > 1 (nccl = RCCL over xGMI).  gloo rehearses the "
                         "multi-rank flow on fewer GPUs than ranks (ranks share the visible GPUs "
                         "round-robin; the rate is then not a scaling number)")
    ap.add_argument("--plan", action="store_true",
                    help="print the ranks' shard plan (world, env ranges, seeds) as rank 0's JSON line and exit "
                         "without touching a GPU (checks the launcher and the sharding on CPU)")
    args = ap.parse_args()
    if args.eager:
        args.launch = "events"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `python bench.py --gpus N`: start the N ranks ourselves (before
        # any GPU call) and relay their exit code; rank 0 prints the line
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to print a line for a "
              "different GPU count", file=sys.stderr)
        return 2
    if args.dist_backend == "nccl" and not args.plan:
        visible = visible_gpus()
        if args.gpus > visible:
            print(f"bench.py: --gpus {args.gpus} with RCCL needs {args.gpus} GPUs, {visible} visible",
                  file=sys.stderr)
            return 2
    c = CONFIGS[args.config]
    # this rank's slice [e0, e1) of the global env batch; every device random
    # stream is keyed by the global env id (marlcov.shards), so env e runs the
    # same trajectory whatever the number of GPUs
    from marlcov.shards import shard_range, weak_range
    if args.global_envs:
        e0, e1 = shard_range(args.global_envs, world, rank)
        scaling = "strong"
    else:
        e0, e1 = weak_range(args.envs or c["envs"], rank)
        scaling = "weak"
    B = e1 - e0
    total_envs = args.global_envs or B * world
    if args.maxsteps is None:
        args.maxsteps = c.get("maxsteps", 1000)
    if args.plan:
        return print_plan(args, world, rank, e0, e1, total_envs, scaling)

    cpu = None
    if rank == 0 and world == 1 and args.gpus == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.config, args.cpu_procs, args.cpu_secs)

    if args.sync == "spin":
        set_spin_sync(local)

    import torch
    import torch.distributed as dist

    import marlcov
    from marlcov.shards import aggregate_rate, reduce_run, shard_seeds

    if args.dist_backend == "gloo":
        local %= max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    run = dict(e0=e0, total_envs=total_envs, scaling=scaling,
               rehearsal=world > 1 and args.dist_backend == "gloo")
    if c.get("env") == "super":
        return bench_super(args, c, B, cpu, world, rank, dev, run)
    cfg = dict(BASE, numrobot=c["numrobot"], sensor_config=c["sensor_config"], allow_even_beams=True,
               maxsteps=args.maxsteps, **c.get("extra", {}))
    dj = bool(cfg.get("dijkstra_input"))
    dr = bool(cfg.get("dist_reward"))
    N = c["numrobot"]
    seeds = shard_seeds(e0)
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=c["width"], length=c["width"], prob_obst=0.1,
                                                    seed=seeds["grid_seed"], num_grids=B),
                                   device=dev, seed=seeds["env_seed"], auto_reset=True,
                                   env_offset=seeds["env_offset"])
    env.reset()
    K, W = args.steps, args.warmup
    # per-step actions keyed by (global env id, step), staged in HBM before timing
    actions = torch.empty((W + K, B, N), dtype=torch.uint8, device=dev)
    for i in range(W + K):
        env.random_actions(seeds["action_seed"], i, out=actions[i])
    reward_sum = torch.zeros(B, dtype=torch.float64, device=dev)
    episodes = torch.zeros(B, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    rp, dp, op = env.reward.data_ptr(), env.done.data_ptr(), env.obs.data_ptr()

    for i in range(W):
        rc = env.step_raw(actions[i].data_ptr(), rp, dp, op, sp)
        assert rc == 0, env.lib.mc_last_error()
    torch.cuda.synchronize(dev)
    env.check()

    # every launch argument resolved before the timed region
    astride = B * N
    tot0 = env.get_state(marlcov._lib.FIELD_DIST_TOTALS).cpu().tolist() if dr else None
    aptrs = [actions[W + i].data_ptr() for i in range(K)]
    a0 = aptrs[0] if K else 0
    elapsed, kern_ms, issue_us = timed_launches(
        lambda i, st: env.step_raw(aptrs[i], rp, dp, op, st), dev, K, args.launch,
        many_call=lambda st: native_call(env, a0, astride, K, rp, dp, op, st),
        first_call=lambda st: (native_call(env, a0, astride, 1, rp, dp, op, st),
                               native_call(env, a0 + astride, astride, K - 1, rp, dp, op, st)),
        events=args.events)
    env.check()
    listed = dj_listed = served = dtot = None
    if dr:  # maps the last step sent to the full distance transform, and those the cache served (diagnostic)
        listed = int(env.get_state(marlcov._lib.FIELD_DIST_LISTED).item())
        served = int(env.get_state(marlcov._lib.FIELD_DIST_CACHED).item())
        tot1 = env.get_state(marlcov._lib.FIELD_DIST_TOTALS).cpu().tolist()
        dtot = dict(zip(("listed", "served", "full", "launches"), (b - a for a, b in zip(tot0, tot1))))
    if dj:  # (env, agent) paths the last step sent to the full-map BFS (diagnostic)
        dj_listed = int(env.get_state(marlcov._lib.FIELD_DJ_LISTED).item())

    # scalar episode-return statistics: the only collective (outside timing)
    reward_sum += env.reward
    episodes += env.done.to(torch.float64)
    stats = torch.stack([reward_sum.sum(), episodes.sum()])
    stats, elapsed = reduce_run(stats, elapsed, world)

    n_gpus = world
    value = aggregate_rate(total_envs, K, elapsed)
    kern_from = KERNEL_US_FROM[args.launch]
    if args.launch == "native" and args.events != "around":
        if kern_ms is None:  # --events none: no events in the timed region
            kern_ms = elapsed / K * 1e3
            kern_from = "no events in the timed region (--events none): wall time per step"
        else:
            kern_from = ("HIP events after the first launch (its own mc_step_many call) and after the last: "
                         "the K - 1 later launches / (K - 1) (includes kernel boundaries)")
    # §8(d): C5's float32 distance layer is 4 B per cell (100 B per agent at
    # E=5) and its two transforms read the whole bit map
    bpe = algorithmic_bytes_per_env_step(N, c["sensor_config"]["range"], cfg["egoradius"],
                                         layers=3 + (4 if dr else 0) + (1 if dj else 0),
                                         full_map_cells=(c["width"] + 2 + 2 * cfg["egoradius"]) ** 2
                                         if dr else (DJ_WINDOW_CELLS if dj else 0))
    achieved = bpe * B / (kern_ms * 1e-3) / 1e9
    design = None
    if dr:
        # the honest C5 price: the windowed 8(d) bytes plus the full-map
        # reads / cache reads the timed steps really made;
        # 8(d)'s full-map figure stays as a labelled upper-bound price
        ext = c["width"] + 2 + 2 * cfg["egoradius"]
        dbytes = c5_design_bytes_per_step(B, N, c["sensor_config"]["range"], cfg["egoradius"], ext,
                                          dtot["listed"], dtot["served"], dtot["full"], dtot["launches"])
        upper = achieved
        achieved = dbytes / (kern_ms * 1e-3) / 1e9
        design = {"design_bytes_per_step": round(dbytes), "design_bytes_per_env_step": round(dbytes / B, 1),
                  "timed_dist_totals": {**dtot, "per_step": {k: round(v / max(1, dtot["launches"]), 1)
                                                             for k, v in dtot.items() if k != "launches"}},
                  "achieved_from": "design bytes (windowed 8(d) part + the full-map and cache reads the timed "
                                   "steps made, MC_FIELD_DIST_TOTALS) / kernel_us",
                  "upper_bound_price": {"bytes_per_env_step": bpe, "achieved": round(upper, 2),
                                        "frac": round(upper / HBM_PEAK_GBS, 5),
                                        "note": "SURVEY 8(d) prices a full-map read per agent and step; the "
                                                "witness test and the top-cell cache skip most of them, so this "
                                                "is not the work timed"}}
    traffic = load_traffic(args.config)
    measured = measured_traffic(args.config, W, K)
    line = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "env-steps/s",
        "n_gpus": n_gpus,
        "steps": K,
        "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 5),
        "higher_is_better": True,
        "scaling": None if run["rehearsal"] else run["scaling"],
        "vs_baseline": None,
        "dtype": "f64+u64",
        "data": "synthetic (device Bernoulli p_obst=0.1 grids, uniform random actions; Philox keyed by "
                "global env id)",
        "config": {"workload": c["desc"], "envs_per_gpu": B, "global_envs": total_envs,
                   "launch": LAUNCH_DESC[args.launch], "host_issue_us_per_step": issue_us,
                   "host_sync": args.sync, "timing_events": args.events,
                   "kernel_variant": env.kernel_variant(),
                   **dist_desc(args, world),
                   "parallelism": f"env-shard x{n_gpus}", "auto_reset": True, "maxsteps": args.maxsteps,
                   "episode_phase": f"timed steps {W + 1}..{W + K} after the first reset (auto-reset at maxsteps)",
                   **({"dist_listed_maps_last_step": listed, "dist_cache_served_last_step": served} if dr else {}),
                   **({"dijkstra_full_map_paths_last_step": dj_listed} if dj else {})},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": traffic,
                     "kernel": "mc::env_kernel" + (" + mc::dijkstra_window_kernel + mc::dijkstra_kernel (one step)"
                                                   if dj else " + the distance kernels (one step)" if dr else ""),
                     "kernel_us": round(kern_ms * 1e3, 3),
                     "kernel_us_from": kern_from + (" (every kernel of a step)" if dj or dr else ""),
                     "alg_bytes_per_env_step": bpe,
                     "achieved_from": "SURVEY 8(d) algorithmic bytes x envs / kernel_us",
                     "measured_traffic": measured,
                     **(design or {})},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def visible_gpus():
    """HIP devices this process may use (torch.cuda.device_count() does not
    initialise the GPU on this image, so the launcher can call it)."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(args):
    """`python bench.py --gpus N` without torchrun: run N ranks as a CHILD
    `python -m torch.distributed.run --nproc-per-node N bench.py <same args>`
    (this process never touches the GPU, so no exec after GPU init), relay
    the child's exit code.  Rank 0 prints the JSON line to the inherited
    stdout.  With RCCL, N above the visible GPU count is an error here, not a
    line for fewer GPUs."""
    import socket
    import subprocess
    if args.dist_backend == "nccl" and not args.plan:
        visible = visible_gpus()
        if args.gpus > visible:
            print(f"bench.py: --gpus {args.gpus} with RCCL needs {args.gpus} GPUs, {visible} visible",
                  file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *sys.argv[1:]]
    sys.stdout.flush()
    # relay rank 0's JSON line on stdout, line by line as it comes; anything
    # else the ranks print there (gloo's connection messages) goes to stderr
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        (sys.stdout if line.startswith("{") else sys.stderr).flush()
    return p.wait()


def print_plan(args, world, rank, e0, e1, total_envs, scaling):
    """--plan: every rank's shard (env range and the seeds keyed by its global
    env offset) gathered to rank 0, printed as one JSON line; no GPU work."""
    from marlcov.shards import shard_seeds
    mine = {"rank": rank, "env_range": [e0, e1], "seeds": shard_seeds(e0)}
    plans = [mine]
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        plans = [None] * world
        dist.all_gather_object(plans, mine)
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"plan": plans, "n_gpus": world, "global_envs": total_envs, "scaling": scaling,
                          "config": args.config, "dist_backend": args.dist_backend}), flush=True)
    return 0


def set_spin_sync(local):
    """hipDeviceScheduleSpin on this rank's device, before torch creates its
    context (a no-op flag for the work itself: the host's wait for the last
    kernel spins instead of yielding)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_int(0)
    assert hip.hipGetDeviceCount(ctypes.byref(n)) == 0
    assert hip.hipSetDevice(ctypes.c_int(local % max(1, n.value))) == 0
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    assert rc == 0, f"hipSetDeviceFlags: {rc}"


def dist_desc(args, world):
    """Process-group facts for the config: the backend and the GPUs the ranks
    really ran on (a gloo rehearsal shares fewer GPUs between its ranks: its
    rate is not a scaling number, and the line says so)."""
    import torch
    if world == 1:
        return {}
    phys = torch.cuda.device_count()
    d = {"dist_backend": "rccl" if args.dist_backend == "nccl" else "gloo", "physical_gpus": min(world, phys)}
    if args.dist_backend == "gloo":
        d["rehearsal"] = (f"{world} ranks over {min(world, phys)} visible GPU(s), gloo process group: "
                          "multi-rank flow check, not a scaling measurement")
    return d


def native_call(env, a0, astride, K, rp, dp, op, stream_ptr):
    """mc_step_many's K launches as a zero-argument call with every ctypes
    argument converted beforehand (no Python marshalling between the first
    event record and the first launch)."""
    import ctypes
    f = env.lib.mc_step_many
    vp, i64 = ctypes.c_void_p, ctypes.c_int64
    args = (env._h if isinstance(env._h, vp) else vp(env._h), vp(a0), i64(astride), ctypes.c_int32(K), vp(rp), i64(0),
            vp(dp), i64(0), vp(op), i64(0), None, i64(0), vp(stream_ptr))
    return lambda: f(*args)


def timed_launches(step_fn, dev, K, launch, many_call=None, first_call=None, events="around"):
    """Time K launches between barrier + synchronize; returns (elapsed s, ms
    per launch from HIP events on the launch stream, host issue time per
    step in us: from the first event record to the last launch returned).

    launch = "native": one C-ABI call issues the K launches (many_call(stream)
    returns the prepared mc_step_many call: one env-kernel launch per step,
    no Python or ctypes per step); its timing events are raw HIP events
    recorded through ctypes (torch's Event.record adds ~8 us of Python and a
    device guard between the first record and the first launch,
    profiles/r5/short_form/).  "stream": the K launches are issued back to back on the stream
    (asynchronous; the host stays ahead of a ~10 us kernel, so the GPU runs
    them back to back and the first kernel starts at once).  "graph": they
    are captured into hipGraphs (chunks of 100) that are instantiated and
    uploaded (hipGraphUpload) before timing, then replayed.  "events": stream
    launches, each bracketed by its own pair of HIP events (per-kernel time;
    the event packets sit between the kernels)."""
    import ctypes

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    stream = torch.cuda.current_stream(dev)
    if launch == "native":
        if events == "after-first" and K > 1:
            c1, c2 = first_call(stream.cuda_stream)
            return timed_native(c2, dev, K, stream, world, first=c1)
        return timed_native(many_call(stream.cuda_stream), dev, K, stream, world, events=events != "none")
    graphs = []
    if launch == "graph":
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        chunk = max(1, min(100, K))
        for c0 in range(0, K, chunk):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                cs = torch.cuda.current_stream(dev).cuda_stream
                for i in range(c0, min(K, c0 + chunk)):
                    step_fn(i, cs)
            graphs.append(g)
            assert hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()),
                                      ctypes.c_void_p(stream.cuda_stream)) == 0
        torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    evs = [ev0, ev1]
    if launch == "events":
        starts = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(K)]
        evs += starts + ends
    # torch creates a HIP event at its first record: do that here, outside the
    # timed region (an event created inside it costs ~tens of us of host time
    # before the first launch)
    for ev in evs:
        ev.record(stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    if launch == "graph":
        for g in graphs:
            g.replay()
    elif launch == "events":
        for i in range(K):
            starts[i].record(stream)
            step_fn(i, stream.cuda_stream)
            ends[i].record(stream)
    else:
        for i in range(K):
            step_fn(i, stream.cuda_stream)
    t_issue = time.perf_counter()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    issue_us = round((t_issue - t0) / K * 1e6, 3)
    if launch == "events":
        return t1 - t0, sum(s_.elapsed_time(e_) for s_, e_ in zip(starts, ends)) / K, issue_us
    return t1 - t0, ev0.elapsed_time(ev1) / K, issue_us


def timed_native(call, dev, K, stream, world, first=None, events=True):
    """The native timed region: raw HIP events (ctypes) around one
    mc_step_many call, between barrier + synchronize on both sides.  With
    `first` (a 1-launch call issued before `call`, whose K - 1 launches the
    events bracket) the first kernel has no marker packet ahead of it, and
    the per-kernel time excludes its start from an idle queue; without
    `events` the region holds the launches alone (per-kernel time None)."""
    import ctypes

    import torch
    import torch.distributed as dist

    hip = ctypes.CDLL("libamdhip64.so")
    sp = ctypes.c_void_p(stream.cuda_stream)
    ev = [ctypes.c_void_p() for _ in range(2)]
    for e in ev:
        assert hip.hipEventCreate(ctypes.byref(e)) == 0
    rec = hip.hipEventRecord
    rec.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    for e in ev:  # first records outside the timed region
        assert rec(e, sp) == 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    rc0 = 0
    if first is not None:
        rc0 = first()
    if events:
        rec(ev[0], sp)
    rc = call()
    t_issue = time.perf_counter()
    if events:
        rec(ev[1], sp)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    assert rc0 == 0 and rc == 0, (rc0, rc)
    if world > 1:
        dist.barrier()
    per = None
    if events:
        ms = ctypes.c_float(0.0)
        assert hip.hipEventElapsedTime(ctypes.byref(ms), ev[0], ev[1]) == 0
        per = ms.value / (K - 1 if first is not None else K)
    for e in ev:
        hip.hipEventDestroy(e)
    return t1 - t0, per, round((t_issue - t0) / K * 1e6, 3)


KERNEL_US_FROM = {
    "native": "HIP events around the K launches of one mc_step_many call / K (includes kernel boundaries)",
    "stream": "HIP events around the K back-to-back launches / K (includes kernel boundaries)",
    "graph": "HIP events around the replayed launches / K (includes kernel boundaries)",
    "events": "per-launch HIP events",
}
LAUNCH_DESC = {"native": "one env-kernel launch per step, the K launches issued by one mc_step_many call",
               "stream": "back-to-back stream launches (one Python/ctypes mc_step call per step)", "graph": "hipGraph replay (uploaded)",
               "events": "stream launches with per-launch events"}


def bench_super(args, c, B, cpu, world, rank, dev, run):
    """SuperGridRL workload: one step = sg_step_kernel +
    sg_dist_kernel over every env of this GPU's shard."""
    import torch
    import torch.distributed as dist

    import marlcov
    from marlcov.shards import aggregate_rate, reduce_run, shard_seeds

    N, W = c["numrobot"], c["width"]
    cfg = dict(SG_BASE, numrobot=N, **c["sg"])
    seeds = shard_seeds(run["e0"])
    env = marlcov.BatchSuperGridEnv(cfg, B, gen=dict(width=W, length=W, prob_obst=0.1, seed=seeds["grid_seed"],
                                                     num_grids=B),
                                    device=dev, seed=seeds["env_seed"], auto_reset=True, maxsteps=args.maxsteps,
                                    env_offset=seeds["env_offset"])
    env.reset()
    K, Wm = args.steps, args.warmup
    g = torch.Generator(device=dev)
    g.manual_seed(seeds["action_seed"] + run["e0"])
    actions = torch.randint(0, 4, (Wm + K, B, N), dtype=torch.uint8, device=dev, generator=g)
    rp, dp = env.reward.data_ptr(), env.done.data_ptr()
    sp = torch.cuda.current_stream(dev).cuda_stream
    for i in range(Wm):
        assert env.step_raw(actions[i].data_ptr(), rp, dp, sp) == 0, env.lib.mc_last_error()
    torch.cuda.synchronize(dev)
    env.check()
    launch = "stream" if args.launch == "native" else args.launch  # (no mc_sg_step_many)
    elapsed, step_ms, issue_us = timed_launches(lambda i, st: env.step_raw(actions[Wm + i].data_ptr(), rp, dp, st),
                                                dev, K, launch)
    env.check()
    stats = torch.stack([env.reward.sum(), env.done.to(torch.float64).sum()])
    stats, elapsed = reduce_run(stats, elapsed, world)
    value = aggregate_rate(run["total_envs"], K, elapsed)
    bpe = sg_algorithmic_bytes_per_env_step(N, cfg["senseradius"], W, W)
    full_dist = os.environ.get("MARLCOV_SG_FULL_DIST") == "1"
    traffic = None if full_dist else load_traffic(args.config)
    if traffic:
        # the distance layer is rewritten only where it changes:
        # the full-refresh bytes would overstate the work, so the achieved
        # bandwidth comes from the measured HBM bytes per step (PMC passes)
        achieved = traffic / (step_ms * 1e-3) / 1e9
        achieved_from = "measured HBM bytes per step (profiles/traffic_sg_c2.json) / step time"
    else:
        achieved = bpe * B / (step_ms * 1e-3) / 1e9
        achieved_from = "full-refresh algorithmic bytes x envs / step time"
    line = {
        "metric": "env-steps/sec (whole node), SuperGridRL 4-agent 128x128 (SURVEY 8(f) rank 2; not the "
                  "BASELINE metric)",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": Wm,
        "ms_per_step": round(elapsed / K * 1e3, 5), "higher_is_better": True,
        "scaling": None if run["rehearsal"] else run["scaling"],
        "vs_baseline": None, "dtype": "f64+u64+f32",
        "data": "synthetic (device Bernoulli p_obst=0.1 grids, uniform random actions)",
        "config": {"workload": c["desc"], "envs_per_gpu": B, "global_envs": run["total_envs"],
                   "launch": LAUNCH_DESC[launch], "host_issue_us_per_step": issue_us,
                   **dist_desc(args, world),
                   "parallelism": f"env-shard x{world}",
                   "auto_reset": True, "maxsteps": args.maxsteps},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "achieved_from": achieved_from,
                     "dist_layer_writes": "whole layer every step" if full_dist else
                                          "changed region (whole layer when max(d) changes)",
                     "kernel": "mcs::sg_step_kernel + mcs::sg_erode_kernel (one step)",
                     "kernel_us": round(step_ms * 1e3, 3),
                     "kernel_us_from": KERNEL_US_FROM[launch] + " (both kernels of a step)",
                     "full_refresh_bytes_per_env_step": bpe},
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
