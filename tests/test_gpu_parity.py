"""GPU parity: the HIP path (libmarlcov.so through its C ABI) against the CPU
oracle and the reference's golden vectors.  Bit-exact on masks, positions,
obs, done and counters; rewards compared exactly (tolerance 0: every reward
term is an integer-valued or config-valued float64 added in reference order,
well inside north_star's 1e-6)."""
import os
import zlib

import numpy as np
import pytest

from golden_util import (KNOWN_ANSWER_POLICIES, case_names, check_against_golden, load_case, load_known_answer,
                         make_env, replay, replay_known_answer)
from gpu_util import compare_env, device_state, oracle_from_device, ref_action
from oracle.cpu_ref import DecGridRLRef

pytestmark = pytest.mark.gpu

REWARD_TOL = 0.0  # north_star allows 1e-6; the build is exact


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def base_cfg(**kw):
    c = dict(numrobot=1, maxsteps=1000, collision_penalty=5, done_thresh=1, done_incr=0,
             terminal_reward=30, dist_reward=0, train_maxsteps=1000, test_maxsteps=1000,
             egoradius=2, mini_map_rad=0, comm_radius=0, allow_comm=0, map_sharing=0,
             single_square_tool=0, dijkstra_input=0, sensor_type="lidar",
             sensor_config={"num_lasers": 21, "range": 10})
    c.update(kw)
    return c


# ---------------------------------------------------------------------------
# 1. the DecGridRL facade replays every golden case of the reference
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", case_names())
def test_facade_matches_reference_golden(torch_cuda, name):
    import marlcov
    case = load_case(name)
    env = make_env(marlcov.DecGridRL, case)
    replay(env, case, check_against_golden(env))


@pytest.mark.parametrize("policy", KNOWN_ANSWER_POLICIES)
def test_facade_known_answer(torch_cuda, policy):
    """SURVEY 8(c) pin 3: the BSA and BA* controllers (Policies/bsa.py:14,
    Policies/ba_star.py:10) cover 100 % of the hand-made test grids
    (Utils/gridmaker.py:23-43; the published result,
    Example_Experiments/Non_Learning/BA_Star/Example/TerminalOutput.txt:
    172-173) with total reward 234 (captured by running the reference in the
    build container, not published).  Their recorded test episodes (captured from the
    reference under the example configs: square sensor r=1,
    single_square_tool, dijkstra_input, egoradius 1) replay through the HIP
    facade with the observation, reward and done of every step equal to the
    record -- so the controllers, deterministic functions of those
    observations, drop in unchanged and reach the same answer."""
    import marlcov
    ka = load_known_answer()
    res = replay_known_answer(marlcov.DecGridRL, ka, policy)
    assert len(res) == 12 and all(r == (234.0, 1.0) for r in res)


# ---------------------------------------------------------------------------
# 2. batched env vs one oracle env per batch entry, random actions
# ---------------------------------------------------------------------------
def full_obs(env, obs, cfg):
    """uint8 obs as float64, with the float32 distance layer in place (the
    reference's z[i][3] when dist_reward is on and dijkstra_input is off)."""
    o = obs.cpu().numpy().astype(np.float64)
    if env.dist_obs is not None and not cfg.get("dijkstra_input"):
        o[:, :, 3] = env.dist_obs.cpu().numpy().astype(np.float64)
    if env.minimap_obs is not None:  # the minimap overwrites layers 3 and 4
        o[:, :, 3:5] = env.minimap_obs.cpu().numpy()
    return o


def bern(rs, w, l, p):
    return rs.choice([1.0, -1.0], size=(w, l), p=[1 - p, p])


def tri(rs, w, l):
    return rs.choice([-1.0, 0.0, 1.0], size=(w, l), p=[0.15, 0.15, 0.7])


BATCH_CASES = {
    # name: (config, grid maker, B, T)
    "c2_like_n4_128": (base_cfg(numrobot=4), lambda rs: bern(rs, 128, 128, 0.1), 12, 30),
    "c4_like_n8_256_360beams": (base_cfg(numrobot=8, allow_even_beams=True,
                                         sensor_config={"num_lasers": 360, "range": 20}),
                                lambda rs: bern(rs, 256, 256, 0.1), 3, 6),
    "nonsquare_70x150_r12": (base_cfg(numrobot=5, sensor_config={"num_lasers": 31, "range": 12}),
                             lambda rs: bern(rs, 70, 150, 0.2), 8, 25),
    "frac_range_float_pen": (base_cfg(numrobot=3, collision_penalty=0.25, terminal_reward=1.5,
                                      sensor_config={"num_lasers": 13, "range": 6.5}),
                             lambda rs: bern(rs, 40, 40, 0.25), 8, 30),
    "zero_cells": (base_cfg(numrobot=3, sensor_config={"num_lasers": 17, "range": 7}),
                   lambda rs: tri(rs, 50, 50), 8, 30),
    "square_r2": (base_cfg(numrobot=3, sensor_type="square_sensor", sensor_config={"range": 2}),
                  lambda rs: tri(rs, 40, 40), 8, 30),
    "square_r1_ego3": (base_cfg(numrobot=2, egoradius=3, sensor_type="square_sensor",
                                sensor_config={"range": 1}),
                       lambda rs: bern(rs, 30, 30, 0.2), 8, 30),
    "single_square_tool": (base_cfg(numrobot=2, single_square_tool=1, sensor_type="square_sensor",
                                    sensor_config={"range": 2}),
                           lambda rs: bern(rs, 30, 30, 0.2), 8, 30),
    # single_square_tool with the lidar: the free map gets only the robot's
    # cell, the obstacle map the lidar's marks (dec_grid_rl.py:232-236)
    "lidar_single_tool": (base_cfg(numrobot=3, single_square_tool=1, sensor_config={"num_lasers": 13, "range": 5}),
                          lambda rs: bern(rs, 30, 30, 0.2), 8, 30),
    "lidar360_single_tool": (base_cfg(numrobot=2, single_square_tool=1, allow_even_beams=True,
                                      sensor_config={"num_lasers": 360, "range": 8}),
                             lambda rs: bern(rs, 40, 40, 0.15), 4, 20),
    "map_sharing_comm": (base_cfg(numrobot=4, comm_radius=7, allow_comm=1, map_sharing=1,
                                  sensor_config={"num_lasers": 15, "range": 5}),
                         lambda rs: bern(rs, 40, 40, 0.15), 8, 30),
    "crowded_n12": (base_cfg(numrobot=12, collision_penalty=2,
                             sensor_config={"num_lasers": 9, "range": 3}),
                    lambda rs: bern(rs, 14, 14, 0.3), 8, 40),
    "done_incr_small": (base_cfg(numrobot=2, done_thresh=0.2, done_incr=0.15, maxsteps=25,
                                 sensor_config={"num_lasers": 11, "range": 4}),
                        lambda rs: bern(rs, 16, 16, 0.1), 8, 40),
    "ego0_range0": (base_cfg(numrobot=2, egoradius=0, sensor_config={"num_lasers": 5, "range": 0}),
                    lambda rs: bern(rs, 12, 12, 0.1), 4, 20),
    "n33_wide_window": (base_cfg(numrobot=33, sensor_config={"num_lasers": 7, "range": 3}),
                        lambda rs: bern(rs, 30, 30, 0.1), 2, 10),
    # the accepted maxima (DESIGN.md §7 limits): 64 robots; lidar range 27
    # (8 x 8 window tiles, 64-bit march rows) with egoradius 15
    "limit_n64_agents": (base_cfg(numrobot=64, collision_penalty=1.5,
                                  sensor_config={"num_lasers": 7, "range": 3}),
                         lambda rs: bern(rs, 40, 40, 0.1), 2, 12),
    "limit_range27_ego15": (base_cfg(numrobot=4, egoradius=15, sensor_config={"num_lasers": 13, "range": 27}),
                            lambda rs: bern(rs, 90, 70, 0.1), 2, 10),
    # dense beam sets: the fan march (sectors of adjacent beams, mc_env_kernel
    # fan_march) on 64-bit rows with special beams, without special beams at
    # range 27, and on 32-bit rows (window of 3 x 3 tiles)
    "fan_128beams_r13_nonsquare": (base_cfg(numrobot=3, allow_even_beams=True,
                                            sensor_config={"num_lasers": 128, "range": 13.5}),
                                   lambda rs: bern(rs, 60, 90, 0.12), 6, 25),
    "fan_361beams_r27": (base_cfg(numrobot=2, sensor_config={"num_lasers": 361, "range": 27}),
                         lambda rs: bern(rs, 80, 80, 0.08), 3, 10),
    "fan_100beams_r6_u32": (base_cfg(numrobot=3, allow_even_beams=True,
                                     sensor_config={"num_lasers": 100, "range": 6}),
                            lambda rs: bern(rs, 40, 40, 0.15), 6, 30),
    # dijkstra_input obs layer: BFS path to the nearest
    # unexplored cell; long episodes on small grids reach long paths
    "dijkstra_square_r1": (base_cfg(numrobot=2, dijkstra_input=1, sensor_type="square_sensor",
                                    sensor_config={"range": 1}, egoradius=2),
                           lambda rs: bern(rs, 20, 20, 0.15), 8, 80),
    "dijkstra_lidar_n3": (base_cfg(numrobot=3, dijkstra_input=1,
                                   sensor_config={"num_lasers": 9, "range": 4}),
                          lambda rs: tri(rs, 36, 28), 8, 60),
    "dijkstra_c2_like": (base_cfg(numrobot=4, dijkstra_input=1), lambda rs: bern(rs, 128, 128, 0.1),
                         4, 12),
    # the BFS window (64 x 64 around the robot's tile) against tiny and wide
    # maps, a 12-cell pad ring (targets in the ring) and a 25-cell crop
    "dijkstra_ego12_tiny": (base_cfg(numrobot=2, dijkstra_input=1, egoradius=12,
                                     sensor_config={"num_lasers": 7, "range": 3}),
                            lambda rs: bern(rs, 9, 7, 0.15), 6, 30),
    "dijkstra_wide_40x150": (base_cfg(numrobot=3, dijkstra_input=1,
                                      sensor_config={"num_lasers": 9, "range": 4}),
                             lambda rs: tri(rs, 40, 150), 4, 40),
    # dist_reward: float32 distance terms in the reward and
    # the float obs layer; with dijkstra_input too the path overwrites it
    "dist_lidar_n3": (base_cfg(numrobot=3, dist_reward=1, sensor_config={"num_lasers": 15, "range": 5}),
                      lambda rs: bern(rs, 30, 26, 0.15), 6, 40),
    "dist_square_ego3": (base_cfg(numrobot=2, dist_reward=1, egoradius=3, sensor_type="square_sensor",
                                  sensor_config={"range": 2}), lambda rs: tri(rs, 22, 22), 6, 40),
    "dist_and_dijkstra": (base_cfg(numrobot=2, dist_reward=1, dijkstra_input=1,
                                   sensor_config={"num_lasers": 9, "range": 4}),
                          lambda rs: bern(rs, 20, 20, 0.1), 6, 40),
    "dist_c5_like_n16": (base_cfg(numrobot=16, dist_reward=1), lambda rs: bern(rs, 64, 64, 0.1), 2, 6),
    # wide, short grids: the witness column passes 4096 (the transform's
    # packed max key keeps 16 bits per field)
    "dist_wide_short": (base_cfg(numrobot=2, dist_reward=1, sensor_config={"num_lasers": 9, "range": 4}),
                        lambda rs: bern(rs, 30, 4200, 0.1), 4, 20),
    # long episodes: max(d) drops many times (the env kernel's witness test
    # sends those maps to the full transform, the rest keep M and take their
    # targets from the window search); single_square_tool keeps coverage thin
    # and max(d) large
    "dist_long_walk": (base_cfg(numrobot=4, dist_reward=1, sensor_config={"num_lasers": 9, "range": 3}),
                       lambda rs: bern(rs, 40, 40, 0.1), 6, 150),
    "dist_single_tool": (base_cfg(numrobot=3, dist_reward=1, single_square_tool=1, sensor_type="square_sensor",
                                  sensor_config={"range": 1}), lambda rs: bern(rs, 36, 44, 0.1), 4, 120),
    # map sharing changes the maps at the start of a step: the PRE transform
    # runs again instead of reusing the previous step's POST data
    "dist_map_sharing": (base_cfg(numrobot=4, dist_reward=1, comm_radius=6, allow_comm=1, map_sharing=1,
                                  sensor_config={"num_lasers": 11, "range": 4}),
                         lambda rs: bern(rs, 30, 30, 0.15), 6, 30),
    # minimap layers (mini_map_rad > 0): the template
    # config's shape, down-scales with dist / dijkstra underneath, up-scale,
    # equal sizes (cv::resize copies)
    "minimap_ego5_mini10_comm": (base_cfg(numrobot=3, egoradius=5, mini_map_rad=10, comm_radius=10,
                                          allow_comm=1, map_sharing=1, sensor_config={"num_lasers": 21, "range": 6}),
                                 lambda rs: bern(rs, 40, 40, 0.15), 6, 30),
    "minimap_dist_dijkstra": (base_cfg(numrobot=2, mini_map_rad=7, dist_reward=1, dijkstra_input=1,
                                       sensor_config={"num_lasers": 11, "range": 4}),
                              lambda rs: tri(rs, 30, 30), 6, 30),
    "minimap_upscale": (base_cfg(numrobot=2, egoradius=4, mini_map_rad=2, sensor_type="square_sensor",
                                 sensor_config={"range": 1}), lambda rs: bern(rs, 20, 20, 0.1), 6, 30),
    "minimap_equal_sizes": (base_cfg(numrobot=2, egoradius=3, mini_map_rad=3), lambda rs: bern(rs, 24, 24, 0.1),
                            4, 20),
}


# dense beam sets: the lidar marches by sectors (fan_march) unless
# MARLCOV_FAN=0 / MARLCOV_BEAM_TABLE keep the ray march
FAN_CASES = sorted([n for n in BATCH_CASES if n.startswith("fan_")] +
                   ["c4_like_n8_256_360beams", "lidar360_single_tool"])


@pytest.mark.parametrize("name", sorted(BATCH_CASES))
def test_batch_matches_oracle(torch_cuda, name):
    import marlcov
    torch = torch_cuda
    cfg, maker, B, T = BATCH_CASES[name]
    rs = np.random.RandomState(zlib.crc32(name.encode()))
    grids = [maker(rs) for _ in range(B)]
    N = cfg["numrobot"]
    refs, pos = [], []
    for b in range(B):
        np.random.seed(1000 + b)
        r = DecGridRLRef([grids[b]], cfg)
        refs.append(r)
        pos.append(np.stack([r._xinds, r._yinds], 1))
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=False, want_adjacency=True)
    if name in FAN_CASES:
        want = os.environ.get("MARLCOV_FAN") != "0" and "MARLCOV_BEAM_TABLE" not in os.environ
        assert ("+fan(" in env.kernel_variant()) == want, env.kernel_variant()
    obs, adj = env.reset(positions=np.stack(pos))
    st = device_state(env)
    obs_h = full_obs(env, obs, cfg)
    for b in range(B):
        compare_env(st, b, refs[b], f"{name} reset env {b}")
        np.testing.assert_array_equal(obs_h[b], refs[b].get_egocentric_observations(),
                                      err_msg=f"{name} reset obs {b}")
    for t in range(T):
        acts = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
        acts[rs.rand(B, N) < 0.08] = rs.choice([4, 7, 200])
        acts[rs.rand(B) < 0.05, 0] = 255
        (obs, adj), rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h, adj_h = (full_obs(env, obs, cfg), rew.cpu().numpy(),
                                       done.cpu().numpy(), adj.cpu().numpy())
        st = device_state(env)
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"{name} t={t} env {b}"
            assert abs(float(r) - rew_h[b]) <= REWARD_TOL, (tag, float(r), rew_h[b])
            assert bool(d) == bool(done_h[b]), tag
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            np.testing.assert_array_equal(adj_h[b], refs[b]._adjacency_matrix, err_msg=tag + " adj")
            compare_env(st, b, refs[b], tag)
        if cfg.get("dist_reward"):
            check_dist_mw(env, refs, f"{name} t={t}")
    env.check()


def check_dist_mw(env, refs, tag, envs=None):
    """Every known (M, witness) of the device equals the oracle's fresh
    distance transform: M = its max, d(witness) = M.  ``refs``: a list (env
    b = refs[b]) or a dict {b: oracle env}."""
    from marlcov import _lib
    from oracle.cpu_ref import l1_distance_to_covered
    mw = env.get_state(_lib.FIELD_DIST_MW).cpu().numpy()
    known = 0
    items = refs.items() if isinstance(refs, dict) else enumerate(refs)
    for b, ref in items:
        p = ref._pad
        for i in range(ref._numrobot):
            M, w = int(mw[b, i, 0]), int(mw[b, i, 1])
            if M < 0:
                continue
            known += 1
            d = l1_distance_to_covered(ref._free_pad[i])
            wx, wy = w >> 16, ((w & 0xFFFF) ^ 0x8000) - 0x8000
            assert M == int(d.max()), (tag, b, i, M, d.max())
            assert int(d[wx + p, wy + p]) == M, (tag, b, i, "witness", wx, wy)
    assert known > 0, tag


# ---------------------------------------------------------------------------
# 3. auto-reset: done envs restart in the same launch; the new episode equals
#    the oracle's reset at the device-drawn start cells
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dist", [0, 1])
def test_auto_reset_matches_oracle_reset(torch_cuda, dist):
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=3, maxsteps=6, dist_reward=dist, sensor_config={"num_lasers": 11, "range": 4})
    rs = np.random.RandomState(7)
    B = 16
    grids = [bern(rs, 24, 24, 0.2) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=True, seed=123)
    env.reset()
    st = device_state(env)
    refs = [oracle_from_device(st, b, cfg) for b in range(B)]
    resets = 0
    from marlcov import _lib
    for t in range(20):
        acts = rs.randint(0, 4, size=(B, 3)).astype(np.uint8)
        acts[rs.rand(B) < 0.08, 0] = 255  # a sentinel's done resets the env too
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env)
        ep_pc = env.get_state(_lib.FIELD_EP_PC).cpu().numpy()
        ep_len = env.get_state(_lib.FIELD_EP_LEN).cpu().numpy()
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            assert float(r) == rew_h[b] and bool(d) == bool(done_h[b]), (t, b)
            if d:
                # the episode record: utils.py:141's percent_covered() and the length
                assert ep_pc[b] == refs[b].percent_covered() and ep_len[b] == refs[b]._currstep, (t, b)
                resets += 1
                p = st["pos"][b]
                assert len({tuple(q) for q in p}) == 3
                for x, y in p:
                    assert refs[b]._grid[x, y] >= 0
                o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in p])
                assert int(st["currstep"][b]) == 0
            np.testing.assert_array_equal(obs_h[b], o, err_msg=f"t={t} env {b}")
            compare_env(st, b, refs[b], f"t={t} env {b}")
    assert resets >= B  # maxsteps=6 over 20 steps: every env reset at least once
    env.check()


# ---------------------------------------------------------------------------
# 4. BASELINE configs[1] at full size (4096 envs, 4 agents, 128x128, lidar
#    21/10): size-independent invariants every step, plus oracle parity of a
#    sample of envs re-built from device state mid-run
# ---------------------------------------------------------------------------
def popcount_rows(bits):
    return bits.reshape(bits.shape[0], -1).sum(axis=1)


def test_c2_full_size_invariants_and_sampled_parity(torch_cuda):
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=4)
    B = 4096
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=128, length=128, prob_obst=0.1, seed=1000),
                                   seed=5, auto_reset=True)
    env.reset()
    g = torch.Generator(device=env.device)
    g.manual_seed(0)
    for t in range(60):
        acts = torch.randint(0, 4, (B, 4), dtype=torch.uint8, device=env.device, generator=g)
        obs, rew, done = env.step(acts)
    torch.cuda.synchronize()
    env.check()
    st = device_state(env)
    # invariants (every env)
    neg = st["neg"][st["env_grid"]]
    assert not np.any(st["free"] & neg[:, None]), "free cell on an obstacle"
    assert not np.any(st["obst"] & (1 - neg[:, None])), "obstacle mark on a free cell"
    union = st["free"].max(axis=1)
    np.testing.assert_array_equal(union, st["vis"])
    np.testing.assert_array_equal(popcount_rows(st["free"]), st["free_cnt"])
    np.testing.assert_array_equal(popcount_rows(st["vis"]), st["vis_cnt"])
    p = st["pos"]
    for b in range(0, B, 97):
        assert len({tuple(q) for q in p[b]}) == 4
    assert np.all(neg[np.arange(B)[:, None], p[..., 0], p[..., 1]] == 0)
    # sampled parity: 24 envs re-built in the oracle, 8 more steps
    sample = np.random.RandomState(3).choice(B, 24, replace=False)
    refs = {b: oracle_from_device(st, b, cfg) for b in sample}
    rs = np.random.RandomState(11)
    for t in range(8):
        acts = rs.randint(0, 4, size=(B, 4)).astype(np.uint8)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env, sample)
        for b in sample:
            o, r, d = refs[b].step(acts[b].astype(np.int64))
            assert float(r) == rew_h[b] and bool(d) == bool(done_h[b]), (t, b)
            if d:  # auto-reset happened on the device: follow it
                q = st["pos"][b]
                o, _ = refs[b].reset(False, None, positions=[tuple(x) for x in q])
            np.testing.assert_array_equal(obs_h[b], o)
            compare_env(st, b, refs[b], f"c2 t={t} env {b}")


def test_determinism_same_seed(torch_cuda):
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=4, maxsteps=20)
    outs = []
    for _ in range(2):
        env = marlcov.BatchCoverageEnv(cfg, 256, gen=dict(width=64, length=64, prob_obst=0.1, seed=9),
                                       seed=77, auto_reset=True)
        env.reset()
        g = torch.Generator(device=env.device)
        g.manual_seed(1)
        acc = []
        for t in range(50):
            acts = torch.randint(0, 4, (256, 4), dtype=torch.uint8, device=env.device, generator=g)
            obs, rew, done = env.step(acts)
            acc.append((obs.clone(), rew.clone(), done.clone()))
        outs.append(acc)
    for (o1, r1, d1), (o2, r2, d2) in zip(*outs):
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2)


# ---------------------------------------------------------------------------
# reset_grid_mode="random": an auto-reset draws a new grid from the pool; the
# new episode equals an oracle reset on that grid at the device-drawn cells
# ---------------------------------------------------------------------------
def test_auto_reset_random_grid_pool(torch_cuda):
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=2, maxsteps=5, sensor_config={"num_lasers": 9, "range": 4})
    rs = np.random.RandomState(31)
    pool = [bern(rs, 20, 20, 0.2) for _ in range(5)]
    B = 12
    env = marlcov.BatchCoverageEnv(cfg, B, grids=pool, auto_reset=True, seed=17, reset_grid_mode="random")
    env.reset()
    st = device_state(env)
    refs = [oracle_from_device(st, b, cfg) for b in range(B)]
    used = set()
    for t in range(30):
        acts = rs.randint(0, 4, size=(B, 2)).astype(np.uint8)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            assert float(r) == rew_h[b] and bool(d) == bool(done_h[b]), (t, b)
            if d:  # a fresh oracle on the grid the device drew, reset at its cells
                g = int(st["env_grid"][b])
                assert 0 <= g < len(pool)
                used.add(g)
                np.random.seed(0)
                refs[b] = DecGridRLRef([pool[g]], cfg)
                o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in st["pos"][b]])
            np.testing.assert_array_equal(obs_h[b], o, err_msg=f"t={t} env {b}")
            compare_env(st, b, refs[b], f"t={t} env {b}")
    assert len(used) >= 4  # the draws cover the pool
    env.check()


@pytest.mark.parametrize("name", ["c2_like_n4_128", "c4_like_n8_256_360beams", "nonsquare_70x150_r12"])
def test_batch_matches_oracle_full_beam_table(torch_cuda, name, monkeypatch):
    """The same cases with the per-start beam table forced on (the march
    otherwise uses each beam's common step bits when the host proves them
    equivalent: mc_set_beam_table, State::beam_common)."""
    monkeypatch.setenv("MARLCOV_BEAM_TABLE", "1")
    test_batch_matches_oracle(torch_cuda, name)


def test_fan_exceptional_starts(torch_cuda):
    """360 beams: 270 and 315 degrees leave their common step pattern from the
    minor starts x = 1..3 (mc_set_beam_table), where the sector march leaves
    them out and marches them alone from the start's own bits.  Robots start
    on rows 1..3 and near the other borders; every step is compared."""
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=4, allow_even_beams=True, sensor_config={"num_lasers": 360, "range": 8})
    rs = np.random.RandomState(360)
    B, N, T = 8, 4, 16
    grids = [bern(rs, 30, 34, 0.1) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=False)
    assert "+fan(" in env.kernel_variant(), env.kernel_variant()
    pos = np.zeros((B, N, 2), np.int32)
    refs = []
    for b in range(B):
        g = np.pad(grids[b], 1, constant_values=-1)
        cells = []
        for x in [1 + b % 3, 2, 3, 30 - b % 3]:  # padded rows 1..3 (exceptional) and the far border
            free = [y for y in range(1, g.shape[1] - 1) if g[x, y] >= 0 and (x, y) not in cells]
            cells.append((x, free[rs.randint(len(free))]))
        pos[b] = cells
        np.random.seed(b)
        r = DecGridRLRef([grids[b]], cfg)
        r.reset(False, None, positions=cells)
        refs.append(r)
    obs = env.reset(positions=pos)
    st = device_state(env)
    for b in range(B):
        compare_env(st, b, refs[b], f"reset env {b}")
    for t in range(T):
        acts = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h = full_obs(env, obs, cfg), rew.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"t={t} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
    env.check()


# dense beam sets over a spread of beam counts, ranges and window widths
# (32- and 64-bit rows, sector sizes 1..6, specials or none): the fan march
# against the oracle
FAN_SWEEP = [(64, 6.0, 2, 24, 30), (96, 9.5, 3, 30, 26), (200, 12.0, 2, 34, 40), (256, 15.0, 4, 50, 44),
             (450, 18.0, 3, 60, 60), (720, 22.0, 2, 70, 64), (361, 25.5, 5, 80, 70), (512, 27.0, 1, 90, 90)]


@pytest.mark.parametrize("nb,rng,n,w,l", FAN_SWEEP, ids=[f"b{c[0]}_r{c[1]}" for c in FAN_SWEEP])
def test_fan_sweep(torch_cuda, nb, rng, n, w, l):
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=n, allow_even_beams=True, sensor_config={"num_lasers": nb, "range": rng})
    rs = np.random.RandomState(nb)
    B, T = 3, 8
    grids = [bern(rs, w, l, 0.12) for _ in range(B)]
    refs, pos = [], []
    for b in range(B):
        np.random.seed(500 + b)
        r = DecGridRLRef([grids[b]], cfg)
        refs.append(r)
        pos.append(np.stack([r._xinds, r._yinds], 1))
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=False)
    assert "+fan(" in env.kernel_variant(), env.kernel_variant()
    env.reset(positions=np.stack(pos))
    st = device_state(env)
    for b in range(B):
        compare_env(st, b, refs[b], f"b{nb} reset env {b}")
    for t in range(T):
        acts = rs.randint(0, 4, size=(B, n)).astype(np.uint8)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h = full_obs(env, obs, cfg), rew.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"b{nb} t={t} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
    env.check()


@pytest.mark.parametrize("name", FAN_CASES)
def test_batch_matches_oracle_ray_march(torch_cuda, name, monkeypatch):
    """The dense cases with the ray march (MARLCOV_FAN=0) instead of the
    sector march."""
    monkeypatch.setenv("MARLCOV_FAN", "0")
    test_batch_matches_oracle(torch_cuda, name)


@pytest.mark.parametrize("name", ["dist_lidar_n3", "dist_long_walk", "dist_single_tool", "dist_map_sharing"])
def test_batch_dist_multi_wave_slot(torch_cuda, name, monkeypatch):
    """dist_reward configs forced onto a 4-wave workgroup (MARLCOV_NT=256) on
    the generic kernel, where every lane reads all agents' PRE terms in the
    reward and dist_window then overwrites them with the POST terms
    (dec_grid_rl.py:222-223,239-240): the waves of a slot must all pass the
    reward before any POST store."""
    monkeypatch.setenv("MARLCOV_NT", "256")
    import marlcov
    cfg, maker, B, _ = BATCH_CASES[name]
    rs = np.random.RandomState(1)
    env = marlcov.BatchCoverageEnv(cfg, B, grids=[maker(rs) for _ in range(B)], auto_reset=False)
    v = env.kernel_variant()
    assert v.startswith("env_kernel<256,1,") and "generic>" in v, v
    del env
    test_batch_matches_oracle(torch_cuda, name)


def test_batch_dist_packed_slots(torch_cuda):
    """dist_reward configs whose envs pack two to a wave (env_kernel<64,2,...>):
    each env slot of the wave appends its listed maps to its own env's shard
    of the full-transform work list (csrc/mc_env_kernel.hip, the slot-masked
    ballot) -- the oracle comparison of every step covers the transform of
    those entries (dec_grid_rl.py:222-223,239-240,260-282)."""
    import marlcov
    packed = []
    for name in ("dist_lidar_n3", "dist_long_walk", "dist_wide_short", "dist_square_ego3"):
        cfg, maker, B, _ = BATCH_CASES[name]
        rs = np.random.RandomState(1)
        env = marlcov.BatchCoverageEnv(cfg, B, grids=[maker(rs) for _ in range(B)], auto_reset=False)
        if env.kernel_variant().startswith("env_kernel<64,2,"):
            packed.append(name)
        del env
    assert packed, "no dist_reward batch case packs two envs per wave"
    for name in packed:
        test_batch_matches_oracle(torch_cuda, name)


@pytest.mark.parametrize("full", [False, True], ids=["window", "full_map"])
def test_dijkstra_far_targets(torch_cuda, monkeypatch, full):
    """dijkstra_input with the nearest unexplored cell 1..300 steps away
    (dijkstra.py:112-187): the window kernel's exact depth (24 layers) and its
    edges, the full-map kernel for the items it lists, robots near the map
    border, and fully explored maps (empty path: the pad ring walled off by
    observed border obstacles).  MARLCOV_DJ_FULL=1 sends every item to the
    full-map kernel."""
    import marlcov
    from marlcov import _lib
    from marlcov.tiles import cells_to_tiles
    torch = torch_cuda
    if full:
        monkeypatch.setenv("MARLCOV_DJ_FULL", "1")
    else:
        monkeypatch.delenv("MARLCOV_DJ_FULL", raising=False)
    cfg = base_cfg(numrobot=3, dijkstra_input=1, sensor_config={"num_lasers": 9, "range": 3})
    rs = np.random.RandomState(11)
    B, N = 10, 3
    grids = [bern(rs, 110, 96, 0.08) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=False)
    env.reset()
    st = device_state(env)
    W, L = env.width, env.length
    X, Y = np.meshgrid(np.arange(W), np.arange(L), indexing="ij")
    depths = [1, 6, 22, 23, 24, 25, 26, 31, 45, 80, 300]
    free = np.zeros((B, N, W, L), np.uint8)
    obst = np.zeros((B, N, W, L), np.uint8)
    for b in range(B):
        neg = st["neg"][st["env_grid"][b]][:W, :L]
        for i in range(N):
            D = depths[(b + 4 * i) % len(depths)]
            x, y = st["pos"][b, i]
            near = (np.abs(X - x) + np.abs(Y - y)) < D
            free[b, i] = near & (neg == 0)
            obst[b, i] = near & (neg == 1)
    vis = free.max(axis=1)

    def put(field, a):
        env.set_state(field, torch.from_numpy(np.ascontiguousarray(a)))

    put(_lib.FIELD_FREE, cells_to_tiles(free, blocks=True).view(np.int64))
    put(_lib.FIELD_OBST, cells_to_tiles(obst, blocks=True).view(np.int64))
    put(_lib.FIELD_VISITED, cells_to_tiles(vis, blocks=True).view(np.int64))
    put(_lib.FIELD_FREE_COUNT, free.reshape(B, -1).sum(1).astype(np.int32))
    put(_lib.FIELD_VISITED_COUNT, vis.reshape(B, -1).sum(1).astype(np.int32))
    st = device_state(env)
    refs = [oracle_from_device(st, b, cfg) for b in range(B)]
    listed = 0
    for t in range(4):
        acts = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        listed = max(listed, int(env.get_state(_lib.FIELD_DJ_LISTED).item()))
        st = device_state(env)
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"far t={t} env {b}"
            assert float(r) == rew_h[b] and bool(d) == bool(done_h[b]), tag
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
    if not full:
        assert listed > 0  # some paths were farther than the window holds
    env.check()
