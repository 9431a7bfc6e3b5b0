"""World-size-2 gloo runs of the multi-GPU path on CPU.

1. The bookkeeping bench.py uses: global seeds, shard ranges, the post-timing
   all-reduces (sum of the episode statistics, max of the elapsed time) and the
   aggregate rate.  The step path itself has no collective.
2. Sharded stepping: each rank steps ITS slice of a global batch of envs —
   grids, start cells and actions drawn from the host restatement of the
   device's Philox streams keyed by global env id (marlcov.streams), envs
   stepped by the CPU oracle — and the gathered trajectories equal a one-rank
   run of the whole batch.  That is the property the device keys its streams
   for: env e's trajectory does not depend on the number of GPUs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import marlcov  # noqa: F401  (package path shim)
from marlcov.shards import (ACTION_SEED, ENV_SEED, GRID_SEED, aggregate_rate, reduce_run, shard_range,
                            shard_seeds, weak_range)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker(rank, world, port, out):
    _init(rank, world, port)
    try:
        stats = torch.tensor([10.0 * (rank + 1), 3.0 + rank], dtype=torch.float64)
        elapsed = 1.0 + 0.5 * rank
        stats, t = reduce_run(stats, elapsed, world)
        e0, e1 = weak_range(4096, rank)
        seeds = shard_seeds(e0)
        gathered = [None] * world
        dist.all_gather_object(gathered, seeds)
        out[rank] = (stats.tolist(), t, aggregate_rate(4096 * world, 200, t), gathered)
    finally:
        dist.destroy_process_group()


def test_two_rank_reduce_and_rate():
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        stats, t, rate, seeds = out[r]
        assert stats == [30.0, 7.0]            # sum over ranks
        assert t == 1.5                        # max over ranks
        assert rate == pytest.approx(4096 * 2 * 200 / 1.5)
        # the same seeds on every rank; the global env offset tells the shards apart
        assert seeds[0]["grid_seed"] == seeds[1]["grid_seed"] == GRID_SEED
        assert seeds[0]["env_seed"] == seeds[1]["env_seed"] == ENV_SEED
        assert seeds[0]["action_seed"] == seeds[1]["action_seed"] == ACTION_SEED
        assert (seeds[0]["env_offset"], seeds[1]["env_offset"]) == (0, 4096)


@pytest.mark.parametrize("n,world", [(32768, 8), (10, 3), (5, 8), (4096, 1)])
def test_shard_ranges_partition(n, world):
    parts = [shard_range(n, world, r) for r in range(world)]
    assert parts[0][0] == 0 and parts[-1][1] == n
    for (a0, a1), (b0, b1) in zip(parts, parts[1:]):
        assert a1 == b0
    sizes = [b - a for a, b in parts]
    assert max(sizes) - min(sizes) <= 1


def test_single_rank_reduce_is_identity():
    stats = torch.tensor([1.0, 2.0], dtype=torch.float64)
    s, t = reduce_run(stats, 0.25, 1)
    assert s.tolist() == [1.0, 2.0] and t == 0.25


# ---------------------------------------------------------------------------
# 2. sharded stepping of a global batch (oracle envs, host Philox streams)
# ---------------------------------------------------------------------------
SHARD_CFG = dict(numrobot=3, maxsteps=5, collision_penalty=5, done_thresh=1, done_incr=0, terminal_reward=30,
                 dist_reward=0, train_maxsteps=1000, test_maxsteps=1000, egoradius=2, mini_map_rad=0,
                 comm_radius=0, allow_comm=0, map_sharing=0, single_square_tool=0, dijkstra_input=0,
                 sensor_type="lidar", sensor_config={"num_lasers": 9, "range": 4})
SHARD_W, SHARD_STEPS = 14, 12


def run_envs(env_ids, steps=SHARD_STEPS):
    """Step global envs ``env_ids`` as the device does in auto-reset mode:
    grid from the gen stream, start cells from the placement stream (episode
    counter per env), actions from the action stream.  Returns per env the
    list of (reward, done, positions) per step."""
    from marlcov.streams import generated_grid, random_actions, start_cells
    from oracle.cpu_ref import DecGridRLRef
    N = SHARD_CFG["numrobot"]
    out = {}
    for e in env_ids:
        grid = generated_grid(GRID_SEED, 0.1, SHARD_W + 2, SHARD_W + 2, e)
        np.random.seed(0)
        ref = DecGridRLRef([grid[1:-1, 1:-1]], SHARD_CFG)
        ep = 1
        ref.reset(False, None, positions=[tuple(q) for q in start_cells(ENV_SEED, e, ep, grid, N)])
        traj = []
        for t in range(steps):
            a = random_actions(ACTION_SEED, [e], t, N)[0].astype(np.int64)
            _, r, d = ref.step(a)
            if d:
                ep += 1
                ref.reset(False, None, positions=[tuple(q) for q in start_cells(ENV_SEED, e, ep, grid, N)])
            traj.append((float(r), bool(d), np.stack([ref._xinds, ref._yinds], 1).tolist()))
        out[e] = traj
    return out


def _shard_worker(rank, world, port, global_envs, out):
    _init(rank, world, port)
    try:
        e0, e1 = shard_range(global_envs, world, rank)
        mine = run_envs(range(e0, e1))
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        if rank == 0:
            merged = {}
            for part in gathered:
                merged.update(part)
            out["merged"] = merged
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_episodes_match_one_batch():
    global_envs, world = 5, 2
    out = mp.Manager().dict()
    mp.spawn(_shard_worker, args=(world, _free_port(), global_envs, out), nprocs=world, join=True)
    merged = out["merged"]
    whole = run_envs(range(global_envs))
    assert sorted(merged) == list(range(global_envs))
    for e in range(global_envs):
        assert merged[e] == whole[e], e
    # the episodes really ended and restarted inside the run (maxsteps=5)
    assert all(sum(d for _, d, _ in whole[e]) >= 2 for e in whole)


# ---------------------------------------------------------------------------
# 3. bench.py --gpus N starts its own ranks (no torchrun in the command)
# ---------------------------------------------------------------------------
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert all(ln.startswith("{") for ln in lines), p.stdout  # stdout carries the JSON line only
    return p.returncode, [json.loads(ln) for ln in lines], p.stderr


@pytest.mark.parametrize("gpus,config,per_rank", [(2, "c2", 4096), (8, "c2", 4096), (2, "c5", 8192)])
def test_bench_gpus_flag_launches_ranks(gpus, config, per_rank):
    """`python bench.py --gpus N` (no torchrun) runs N ranks: rank 0's one
    line says n_gpus N, the global batch is N x the per-GPU envs (C3 = 8 x
    4,096, C5 = 8 x 8,192), and every rank's shard starts at its global env
    offset (the seeds the device streams are keyed by)."""
    rc, lines, err = _bench(["--gpus", str(gpus), "--dist-backend", "gloo", "--plan", "--config", config])
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    plan = lines[0]
    assert plan["n_gpus"] == gpus and plan["global_envs"] == gpus * per_rank and plan["scaling"] == "weak"
    assert [p["rank"] for p in plan["plan"]] == list(range(gpus))
    for r, p in enumerate(plan["plan"]):
        assert p["env_range"] == [r * per_rank, (r + 1) * per_rank]
        assert p["seeds"] == shard_seeds(r * per_rank)


def test_bench_refuses_world_mismatch():
    """A world size that differs from --gpus exits non-zero without a line."""
    rc, lines, err = _bench(["--gpus", "2", "--plan"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE=1" in err


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """RCCL ranks need one GPU each: --gpus above the visible count exits
    non-zero in the launcher, before any rank starts (nothing printed)."""
    if torch.cuda.device_count() >= 16:
        pytest.skip("16 GPUs visible")
    rc, lines, err = _bench(["--gpus", "16", "--steps", "1", "--warmup", "0", "--no-cpu"])
    assert rc != 0 and not lines and "visible" in err
