"""World-size-2 gloo run of the multi-GPU bookkeeping on CPU:
independent per-rank seeds, shard ranges, the post-timing all-reduces (sum of
the episode statistics, max of the elapsed time) and the aggregate rate that
bench.py reports.  The step path itself has no collective."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import marlcov
from marlcov.shards import aggregate_rate, rank_seeds, reduce_run, shard_range


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        stats = torch.tensor([10.0 * (rank + 1), 3.0 + rank], dtype=torch.float64)
        elapsed = 1.0 + 0.5 * rank
        stats, t = reduce_run(stats, elapsed, world)
        seeds = rank_seeds(rank)
        gathered = [None] * world
        dist.all_gather_object(gathered, seeds)
        out[rank] = (stats.tolist(), t, aggregate_rate(4096, world, 200, t), gathered)
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
        for k in seeds[0]:                     # every stream differs per rank
            assert seeds[0][k] != seeds[1][k]


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
