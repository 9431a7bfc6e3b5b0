"""Env sharding across GPUs: one process per GPU, each rank owns
an independent batch of envs (its own grids, state, stream and seeds); the step
path has no collective.  The only exchange is after timing: the scalar
episode-return statistics (sum) and the elapsed time (max over ranks) — one
RCCL all-reduce each on GPUs, gloo in the CPU tests.
"""
from __future__ import annotations


def rank_seeds(rank: int) -> dict:
    """Independent streams per rank: grid pool, device Philox, action draw."""
    return {"grid_seed": 1000 + rank, "env_seed": 1 + rank, "action_seed": 12345 + rank}


def shard_range(global_envs: int, world: int, rank: int) -> tuple[int, int]:
    """[start, stop) of rank's envs when a fixed global batch is split (strong
    scaling); the remainder goes to the lowest ranks."""
    base, rem = divmod(global_envs, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def reduce_run(stats, elapsed_s: float, world: int):
    """All-reduce the per-rank [return_sum, episodes] tensor (SUM) and the
    elapsed time (MAX).  Returns (stats, max_elapsed_s)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=stats.device)
    if world > 1:
        dist.all_reduce(stats)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return stats, float(t.item())


def aggregate_rate(envs_per_rank: int, world: int, steps: int, elapsed_s: float) -> float:
    """Whole-job env-steps/s: every rank's envs over the slowest rank's time."""
    return envs_per_rank * world * steps / elapsed_s
