"""GPU parity of the bench workloads at the bench's own batch sizes.

bench.py times C2 at 4,096 envs and C4 / C5 at 8,192 envs.
Multi-wave timing bugs (round 3's LDS race) and the C5 dist bookkeeping (the
list sizes, the split factor and the cache tries' per-workgroup shares all
change with B) live in exactly these shapes, so each test here builds the
env exactly as bench.py does (device Bernoulli grid pool keyed by global env
id, shard_seeds(0), auto-reset, the bench's mc_random_actions stream) and:

* tracks a sample of envs through the oracle (oracle/cpu_ref.py) FROM THE
  RESET, every step, through auto-resets (start cells checked against the
  host Philox restatement, marlcov.streams): the accumulated maps, counters,
  positions, obs, reward and done, not only single transitions;
* checks size-independent invariants over EVERY env on the device
  (dec_grid_rl.py:206-258): free marks only on free cells, obstacle marks
  only on obstacle cells, the union plane = OR of the agents' free planes,
  the counters = popcounts, robots on distinct non-obstacle cells;
* asserts the env-kernel instantiation the bench prints (kernel_variant).
"""
import numpy as np
import pytest

from gpu_util import compare_env, device_state, oracle_from_device
from test_gpu_parity import base_cfg, check_dist_mw, full_obs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def popcount64(torch, x):
    """Per-word popcount of an int64 tensor (SWAR; two's-complement wrap)."""
    m1, m2, m4, h01 = 0x5555555555555555, 0x3333333333333333, 0x0F0F0F0F0F0F0F0F, 0x0101010101010101
    x = x - ((x >> 1) & m1)
    x = (x & m2) + ((x >> 2) & m2)
    x = (x + (x >> 4)) & m4
    return ((x * h01) >> 56) & 0xFF


def device_invariants(torch, env, tag):
    """Invariants of every env's state, evaluated on the device."""
    from marlcov import _lib
    B, N = env.num_envs, env.num_agents
    eg = env.get_state(_lib.FIELD_ENV_GRID).long()
    neg_pool = env.get_state(_lib.FIELD_GRID_NEG)
    vis = env.get_state(_lib.FIELD_VISITED)
    fc = env.get_state(_lib.FIELD_FREE_COUNT).long()
    vc = env.get_state(_lib.FIELD_VISITED_COUNT).long()
    chunk = 1024
    for b0 in range(0, B, chunk):
        b1 = min(B, b0 + chunk)
        free = env.get_state(_lib.FIELD_FREE)[b0:b1]
        obst = env.get_state(_lib.FIELD_OBST)[b0:b1]
        neg = neg_pool[eg[b0:b1]].unsqueeze(1)
        assert not bool((free & neg).any()), f"{tag}: free mark on an obstacle cell"
        assert not bool((obst & ~neg).any()), f"{tag}: obstacle mark on a free cell"
        union = free[:, 0].clone()
        for i in range(1, N):
            union |= free[:, i]
        assert torch.equal(union, vis[b0:b1]), f"{tag}: union plane != OR of the free planes"
        pf = popcount64(torch, free).reshape(b1 - b0, -1).sum(1)
        pv = popcount64(torch, vis[b0:b1]).reshape(b1 - b0, -1).sum(1)
        assert torch.equal(pf, fc[b0:b1]), f"{tag}: free counter != popcount"
        assert torch.equal(pv, vc[b0:b1]), f"{tag}: union counter != popcount"
        del free, obst, neg, union
    # robots: distinct cells, none on an obstacle (grid < 0) cell
    pos = env.get_state(_lib.FIELD_POS).long()
    x, y = pos[..., 0], pos[..., 1]
    trs, tcs = neg_pool.shape[1], neg_pool.shape[2]
    ti, tj = x // 8, y // 8
    idx = ((ti // 4) * tcs + tj // 4) * 16 + (ti % 4) * 4 + (tj % 4)
    words = neg_pool.reshape(neg_pool.shape[0], trs * tcs * 16)[eg[:, None], idx]
    bits = (words >> (8 * (x % 8) + (y % 8))) & 1
    assert not bool(bits.any()), f"{tag}: robot on an obstacle cell"
    key, _ = torch.sort(x * 4096 + y, dim=1)
    assert not bool((key[:, 1:] == key[:, :-1]).any()), f"{tag}: two robots on one cell"


def bench_env(cfgname, maxsteps, rank=0):
    """The env exactly as bench.py main() builds it for this config on rank
    ``rank`` (weak scaling: the shard of global envs [rank*B, (rank+1)*B))."""
    import bench
    import marlcov
    from marlcov.shards import shard_seeds
    c = bench.CONFIGS[cfgname]
    cfg = dict(bench.BASE, numrobot=c["numrobot"], sensor_config=c["sensor_config"], allow_even_beams=True,
               maxsteps=maxsteps, **c.get("extra", {}))
    B = c["envs"]
    seeds = shard_seeds(rank * B)
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=c["width"], length=c["width"], prob_obst=0.1,
                                                    seed=seeds["grid_seed"], num_grids=B),
                                   seed=seeds["env_seed"], auto_reset=True, env_offset=seeds["env_offset"])
    return env, cfg, seeds


def run_full_size(torch, cfgname, maxsteps, steps, sample, variant, inv_every, dist_every=0, rank=0):
    """Bench-shaped env of rank ``rank``'s shard; the sample tracked by the
    oracle from the reset.  The sampled envs' pool grids and start cells are
    checked against the host restatement of the streams at their GLOBAL ids
    (offset + b), so a late rank's shard is the global batch's slice."""
    from marlcov import _lib, streams
    env, cfg, seeds = bench_env(cfgname, maxsteps, rank)
    off = seeds["env_offset"]
    assert env.kernel_variant() == variant, env.kernel_variant()
    B, N = env.num_envs, env.num_agents
    env.reset()
    st = device_state(env, sample)
    refs = {}
    for b in sample:
        g = int(st["env_grid"][b])
        grid = np.where(st["neg"][g] == 1, -1.0, np.where(st["pos_plane"][g] == 1, 1.0, 0.0))
        np.testing.assert_array_equal(grid, streams.generated_grid(seeds["grid_seed"], 0.1, grid.shape[0],
                                                                   grid.shape[1], off + g),
                                      err_msg=f"pool grid {g} at global id {off + g}")
        np.testing.assert_array_equal(st["pos"][b], streams.start_cells(seeds["env_seed"], off + b,
                                                                        int(st["episode"][b]), grid, N),
                                      err_msg=f"reset cells {b}")
        np.random.seed(0)
        from oracle.cpu_ref import DecGridRLRef
        ref = DecGridRLRef([grid[1:-1, 1:-1]], cfg)
        ref.reset(False, None, positions=[tuple(q) for q in st["pos"][b]])
        compare_env(st, b, ref, f"{cfgname} reset env {b}")
        refs[b] = ref
    device_invariants(torch, env, f"{cfgname} reset")
    resets = listed = cached = 0
    for t in range(steps):
        a = env.random_actions(seeds["action_seed"], t)
        obs, rew, done = env.step(a)
        a_h = a.cpu().numpy()
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        if cfg.get("dist_reward"):
            listed += int(env.get_state(_lib.FIELD_DIST_LISTED).item())
            cached += int(env.get_state(_lib.FIELD_DIST_CACHED).item())
        st = device_state(env, sample)
        for b in sample:
            o, r, d = refs[b].step(a_h[b].astype(np.int64))
            tag = f"{cfgname} t={t + 1} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            assert bool(d) == bool(done_h[b]), tag
            if d:
                resets += 1
                p = st["pos"][b]
                want = streams.start_cells(seeds["env_seed"], off + b, int(st["episode"][b]), refs[b]._grid, N)
                np.testing.assert_array_equal(p, want, err_msg=tag + " start cells vs host Philox")
                o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in p])
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
        if dist_every and (t % dist_every == 0 or t == steps - 1):
            check_dist_mw(env, refs, f"{cfgname} t={t + 1}", envs=sample)
        if t % inv_every == inv_every - 1 or t == steps - 1:
            device_invariants(torch, env, f"{cfgname} t={t + 1}")
    env.check()
    return env, resets, listed, cached


@pytest.mark.parametrize("rank", [0, 7])
def test_c2_bench_shape_full_size(torch_cuda, rank):
    """C2 (configs[1], the metric's workload): 4,096 envs, 4 agents, 128x128,
    21 beams R=10; maxsteps 20 so every env auto-resets three times in 64
    steps; 16 envs tracked by the oracle from the reset.  rank 7: the last
    shard of C3 (global envs 28,672..32,767 of 8 x 4,096)."""
    sample = [int(b) for b in np.random.RandomState(2).choice(4096, 16, replace=False)]
    env, resets, _, _ = run_full_size(torch_cuda, "c2", 20, 64, sample, "env_kernel<64,2,u32,C2>", inv_every=8,
                                      rank=rank)
    assert resets >= 3 * len(sample)
    ep = env.get_state(__import__("marlcov")._lib.FIELD_EPISODE)
    assert int(ep.min()) >= 4  # every env of the batch: the first episode + 3 auto-resets


def test_c4_bench_shape_full_size(torch_cuda):
    """C4 (configs[3]): 8,192 envs, 8 agents, 256x256, 360 beams R=20, the fan
    march with its two special beams; maxsteps 15 so every env auto-resets
    (three times in 48 steps); 8 envs tracked by the oracle from the reset,
    invariants over all 8,192 envs."""
    sample = [0, 1, 777, 2048, 4095, 5000, 8000, 8191]
    env, resets, _, _ = run_full_size(torch_cuda, "c4", 15, 48, sample, "env_kernel<256,1,u64,C4> +fan(64/2)",
                                      inv_every=16)
    assert resets >= 3 * len(sample)
    assert int(env.get_state(__import__("marlcov")._lib.FIELD_EPISODE).min()) >= 4


@pytest.mark.parametrize("rank", [0, 7])
def test_c5_bench_shape_full_size(torch_cuda, rank):
    """C5 (configs[4], one GPU's shard): 8,192 envs, 16 agents, 512x512,
    dist_reward, the bench's 2000-step episodes: the early phase, steps 1..30
    after the reset, where the most maps go to the distance transform's list.
    4 envs tracked by the oracle from the reset (float32 distance terms in the
    reward, the float distance obs layer), every known (max d, witness) of
    them against a fresh transform, invariants over all envs; the steps must
    list maps for the full transform and the top-cell cache must serve some
    (dec_grid_rl.py:206-258,260-282).  rank 7: the last shard of C5's
    65,536 envs (global envs 57,344..65,535)."""
    from marlcov import _lib
    sample = [0, 2600, 5555, 8191]
    env, _, listed, cached = run_full_size(torch_cuda, "c5", 2000, 30, sample, "env_kernel<128,1,u32,C5>",
                                           inv_every=10, dist_every=3, rank=rank)
    assert listed > 0 and cached > 0, (listed, cached)
    assert int(env.get_state(_lib.FIELD_CURRSTEP).min()) == 30


def run_deep(torch, cfgname, maxsteps, steps, sample, variant, state_every, dist_every=0):
    """Deep-episode parity: the sample is tracked by the
    oracle from the reset through ``steps`` bench steps, so the accumulated
    state -- every free / obstacle / union mark since the reset, the counters
    and positions -- is checked, not a transition from device state.  Obs,
    done and positions every step; the full maps every ``state_every`` steps
    and at the end (unpacking 16 x 512 x 512 planes per step would dominate).

    dist_reward configs: the oracle's distance term is stateless (observe()
    recomputes the map from the free plane, dec_grid_rl.py:222-223,239-240),
    so the tracker runs with it off between checkpoints (obs layers 0..2
    compared, reward not) and on at every ``dist_every``-th step and the last
    25 steps (reward with the float32 distance terms, the float distance obs
    layer)."""
    from marlcov import streams
    from oracle.cpu_ref import DecGridRLRef
    env, cfg, seeds = bench_env(cfgname, maxsteps)
    assert env.kernel_variant() == variant, env.kernel_variant()
    N = env.num_agents
    dist = bool(cfg.get("dist_reward"))
    sel = torch.tensor(sample, device=env.device)
    env.reset()
    st = device_state(env, sample)
    refs = {}
    for b in sample:
        g = int(st["env_grid"][b])
        grid = np.where(st["neg"][g] == 1, -1.0, np.where(st["pos_plane"][g] == 1, 1.0, 0.0))
        np.random.seed(0)
        ref = DecGridRLRef([grid[1:-1, 1:-1]], cfg)
        ref.reset(False, None, positions=[tuple(q) for q in st["pos"][b]])
        refs[b] = ref
    resets = 0
    for t in range(steps):
        a = env.random_actions(seeds["action_seed"], t)
        obs, rew, done = env.step(a)
        full = dist and ((dist_every and t % dist_every == 0) or t >= steps - 25)
        o_dev = obs.index_select(0, sel).cpu().numpy().astype(np.float64)
        if full:
            o_dev[:, :, 3] = env.dist_obs.index_select(0, sel).cpu().numpy().astype(np.float64)
        rew_h, done_h = rew.index_select(0, sel).cpu().numpy(), done.index_select(0, sel).cpu().numpy()
        a_h = a.index_select(0, sel).cpu().numpy()
        check_state = t % state_every == state_every - 1 or t == steps - 1
        st = device_state(env, sample) if check_state else None
        from marlcov import _lib
        pos = env.get_state(_lib.FIELD_POS).index_select(0, sel).cpu().numpy()
        for k, b in enumerate(sample):
            ref = refs[b]
            if dist:
                ref._dist_r = 1 if full else 0
            o, r, d = ref.step(a_h[k].astype(np.int64))
            tag = f"{cfgname} deep t={t + 1} env {b}"
            if full or not dist:
                assert float(r) == rew_h[k], (tag, float(r), rew_h[k])
            assert bool(d) == bool(done_h[k]), tag
            if d:
                resets += 1
                ep = int(env.get_state(_lib.FIELD_EPISODE)[b].item())
                want = streams.start_cells(seeds["env_seed"], b, ep, ref._grid, N)
                np.testing.assert_array_equal(pos[k], want, err_msg=tag + " start cells vs host Philox")
                o, _ = ref.reset(False, None, positions=[tuple(q) for q in pos[k]])
                if dist and not full:
                    o = o[:, :3]
            np.testing.assert_array_equal(o_dev[k][:, :o.shape[1]], o, err_msg=tag + " obs")
            np.testing.assert_array_equal(pos[k, :, 0], ref._xinds, err_msg=tag + " x")
            np.testing.assert_array_equal(pos[k, :, 1], ref._yinds, err_msg=tag + " y")
            if check_state:
                compare_env(st, b, ref, tag)
    env.check()
    return env, resets


def test_c2_bench_shape_deep_episode(torch_cuda):
    """C2 at the bench's own episode length (maxsteps 1000): 4 envs tracked by
    the oracle from the reset through 1,040 steps -- the whole first episode,
    the auto-reset at step 1000 inside the kernel and 40 steps of the next."""
    env, resets = run_deep(torch_cuda, "c2", 1000, 1040, [5, 1234, 2222, 4090], "env_kernel<64,2,u32,C2>",
                           state_every=50)
    assert resets >= 4


def test_c4_bench_shape_deep_episode(torch_cuda):
    """C4 at 8,192 envs: 1 env tracked by the oracle from the reset through 400
    steps (the fan march's marks accumulated over the episode)."""
    run_deep(torch_cuda, "c4", 1000, 400, [4444], "env_kernel<256,1,u64,C4> +fan(64/2)", state_every=50)


def test_c5_bench_shape_deep_episode(torch_cuda):
    """C5 at 8,192 envs: 1 env tracked by the oracle from the reset through 625
    steps -- the accumulated maps under which test_c5_cache_steady_state_
    matches_oracle starts -- with the distance terms checked every 25 steps and
    in the last 25 (the top-cell cache's steady state)."""
    run_deep(torch_cuda, "c5", 2000, 625, [3001], "env_kernel<128,1,u32,C5>", state_every=100, dist_every=25)
