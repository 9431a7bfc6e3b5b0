"""Env sharding across GPUs: one process per GPU, each rank owns
a contiguous range of the global env batch (its own grids, state and stream);
the step path has no collective.  The only exchange is after timing: the scalar
episode-return statistics (sum) and the elapsed time (max over ranks) — one
RCCL all-reduce each on GPUs, gloo in the CPU tests.

Seeds are global, not per rank: every device random stream (grid pool, start
cells, actions) is keyed by the GLOBAL env / grid id (``env_offset`` of
BatchCoverageEnv), so env e of the global batch follows the same trajectory
whatever the number of GPUs (grid seed = 1000 + env id).
"""
from __future__ import annotations

GRID_SEED = 1000   # pool grid of global env e: Philox(GRID_SEED, e)
ENV_SEED = 1       # start-cell draws: Philox(ENV_SEED, e, episode)
ACTION_SEED = 12345  # synthetic actions: Philox(ACTION_SEED, e, step)


def shard_seeds(env_offset: int) -> dict:
    """The device streams of a shard whose first env is global env
    ``env_offset``: the same seeds on every rank, the offset selects the ids."""
    return {"grid_seed": GRID_SEED, "env_seed": ENV_SEED, "action_seed": ACTION_SEED,
            "env_offset": int(env_offset)}


def shard_range(global_envs: int, world: int, rank: int) -> tuple[int, int]:
    """[start, stop) of rank's envs when a fixed global batch is split (strong
    scaling); the remainder goes to the lowest ranks."""
    base, rem = divmod(global_envs, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def weak_range(envs_per_rank: int, rank: int) -> tuple[int, int]:
    """[start, stop) of rank's envs when every rank holds ``envs_per_rank``
    (weak scaling: the global batch grows with the GPU count)."""
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


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


def aggregate_rate(total_envs: int, steps: int, elapsed_s: float) -> float:
    """Whole-job env-steps/s: every rank's envs over the slowest rank's time."""
    return total_envs * steps / elapsed_s
