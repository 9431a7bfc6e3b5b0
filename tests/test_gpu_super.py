"""GPU parity of the SuperGridRL path (SURVEY §8(f) rank 2,
``Environments/super_grid_rl.py``) through the ``mc_sg_*`` C ABI:

1. the ``SuperGridRL`` facade replays every golden case captured from the
   reference (tests/golden/make_golden_super.py);
2. ``BatchSuperGridEnv`` against one oracle env (oracle/super_ref.py) per
   batch entry over random joint actions, sentinels and motion-penalty
   quotients, including both distance-plane paths (LDS and global scratch);
3. auto-reset with the episode cut, against the oracle's reset at the
   device-drawn cells;
4. the bench workload at full size: plane/bitboard invariants on every env,
   16 sampled envs rebuilt in the oracle and stepped on.
Everything is compared exactly, rewards included (tolerance 0, inside
north_star's 1e-6): the device folds each reward slot in the reference's
order and sums the slots with NumPy's pairwise scheme."""
import zlib

import numpy as np
import pytest

from oracle.super_ref import SuperGridRLRef
from super_golden_util import check_super_golden, load_super_case, make_super_env, replay_super, super_case_names

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def sg_cfg(**kw):
    c = dict(numrobot=1, train_maxsteps=1000, test_maxsteps=1000, collision_penalty=5, senseradius=1,
             free_penalty=0.2, done_thresh=1, done_incr=0, terminal_reward=30, dist_reward=0,
             use_scanning=0)
    c.update(kw)
    return c


# ---------------------------------------------------------------------------
# 1. facade vs the reference's golden vectors
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", super_case_names())
def test_super_facade_matches_reference_golden(torch_cuda, name):
    import marlcov
    case = load_super_case(name)
    env = make_super_env(marlcov.SuperGridRL, case)
    replay_super(env, case, check_super_golden(env))


# ---------------------------------------------------------------------------
# 2./3. batch vs oracle
# ---------------------------------------------------------------------------
def device_state(env):
    from marlcov import _lib
    from marlcov.super_env import unpack_rows
    L = env.length
    return dict(
        planes=env.planes.cpu().numpy(), dist=env.dist.cpu().numpy(),
        pos=env.get_state(_lib.SG_FIELD_POS).cpu().numpy(),
        cov=unpack_rows(env.get_state(_lib.SG_FIELD_COVERED).cpu().numpy(), L),
        obst=unpack_rows(env.get_state(_lib.SG_FIELD_OBST).cpu().numpy(), L),
        cov_cnt=env.get_state(_lib.SG_FIELD_COV_COUNT).cpu().numpy(),
        currstep=env.get_state(_lib.SG_FIELD_CURRSTEP).cpu().numpy(),
        done_thresh=env.get_state(_lib.SG_FIELD_DONE_THRESH).cpu().numpy(),
        a_prev=env.get_state(_lib.SG_FIELD_A_PREV).cpu().numpy(),
        env_grid=env.get_state(_lib.SG_FIELD_ENV_GRID).cpu().numpy(),
        neg=unpack_rows(env.get_state(_lib.SG_FIELD_GRID_NEG).cpu().numpy(), L),
        gpos=unpack_rows(env.get_state(_lib.SG_FIELD_GRID_POS).cpu().numpy(), L),
    )


def compare(st, b, ref, tag):
    state, cur = ref.get_state()
    np.testing.assert_array_equal(st["pos"][b, :, 0], ref._xinds, err_msg=tag + " x")
    np.testing.assert_array_equal(st["pos"][b, :, 1], ref._yinds, err_msg=tag + " y")
    np.testing.assert_array_equal(st["planes"][b], state[:-1], err_msg=tag + " uint8 layers")
    np.testing.assert_array_equal(st["dist"][b].astype(np.float64), state[-1], err_msg=tag + " dist layer")
    np.testing.assert_array_equal(st["cov"][b], (ref._free == 0).astype(np.uint8), err_msg=tag + " covered")
    np.testing.assert_array_equal(st["obst"][b], ref._observed_obstacles.astype(np.uint8), err_msg=tag + " obst")
    assert int(st["cov_cnt"][b]) == np.count_nonzero(ref._free < 1), tag
    assert int(st["currstep"][b]) == cur == ref._currstep, tag
    assert float(st["done_thresh"][b]) == float(ref._done_thresh), tag
    assert int(st["a_prev"][b]) == (-1 if ref.a_prev is None else int(ref.a_prev)), tag


def bernoulli(rs, w, l, p):
    return rs.choice([1.0, -1.0], size=(w, l), p=[1 - p, p])


def tri_valued(rs, w, l):
    return np.clip(rs.choice([0, 1, 255], size=(w, l), p=[0.15, 0.15, 0.7]).astype(float) - 1, -1, 1)


def draw_positions(rs, grid, n):
    free = np.argwhere(grid >= 0)
    pick = rs.choice(len(free), size=n, replace=False)
    return free[pick].astype(np.int32)


BATCH_CASES = {
    "n4_r2_dist": (sg_cfg(numrobot=4, senseradius=2, dist_reward=1), (40, 52), 0.15, 24, 60),
    "scan_n6_r1_dist": (sg_cfg(numrobot=6, use_scanning=1, free_penalty=0.35, dist_reward=1), (33, 33), 0.2, 16, 60),
    "n1_r0": (sg_cfg(senseradius=0, free_penalty=0.0), (20, 20), 0.2, 8, 60),
    "zero_cells_n3_r3": (sg_cfg(numrobot=3, senseradius=3, free_penalty=0.7, dist_reward=1), "tri", None, 12, 50),
    "n16_r2_dist": (sg_cfg(numrobot=16, senseradius=2, free_penalty=0.1, dist_reward=1), (64, 64), 0.1, 8, 30),
    "scan_n40_pairwise_sum": (sg_cfg(numrobot=40, use_scanning=1, free_penalty=0.15, dist_reward=1,
                                     collision_penalty=0.75), (24, 24), 0.1, 6, 30),
    # W + L > 257: the separable sweep kernel instead of the erosion kernel,
    # with its u16 planes in the global scratch / in LDS
    "global_scratch_150x300": (sg_cfg(numrobot=4, senseradius=2, dist_reward=1), (150, 300), 0.1, 4, 25),
    "sweep_lds_200x100": (sg_cfg(numrobot=3, senseradius=2, dist_reward=1), (200, 100), 0.02, 4, 25),
    "erode_open_grid_1x250": (sg_cfg(numrobot=2, senseradius=3, dist_reward=1), (1, 250), 0.0, 4, 60),
    "done_incr_small": (sg_cfg(numrobot=3, senseradius=2, done_thresh=0.3, done_incr=0.25, dist_reward=1),
                        (14, 14), 0.1, 10, 80),
    "r15_wide_window": (sg_cfg(numrobot=2, senseradius=15, free_penalty=0.05, dist_reward=1), (70, 90), 0.1, 4, 20),
    # two row words per row, W = 128 (the bench shape's rows), and an open grid
    "wave_rw2_128x124": (sg_cfg(numrobot=4, senseradius=2, free_penalty=0.1, dist_reward=1), (128, 124), 0.1, 6, 40),
    "wave_rw2_open_100x68": (sg_cfg(numrobot=3, senseradius=3, dist_reward=1), (100, 68), 0.0, 4, 40),
}


# the same cases with the one-lane-per-robot step kernel and with the whole
# distance layer rewritten every step (both read when the handle is created)
ALT_MODES = {"lane_per_robot": {"MARLCOV_SG_ROWS": "0"}, "full_dist_layer": {"MARLCOV_SG_FULL_DIST": "1"}}
ALT_CASES = ["n4_r2_dist", "scan_n6_r1_dist", "zero_cells_n3_r3", "n16_r2_dist", "done_incr_small",
             "wave_rw2_128x124"]


@pytest.mark.parametrize("mode", sorted(ALT_MODES))
@pytest.mark.parametrize("name", ALT_CASES)
def test_super_batch_alt_modes(torch_cuda, monkeypatch, name, mode):
    for k, v in ALT_MODES[mode].items():
        monkeypatch.setenv(k, v)
    test_super_batch_matches_oracle(torch_cuda, name)


@pytest.mark.parametrize("name", sorted(BATCH_CASES))
def test_super_batch_matches_oracle(torch_cuda, name):
    import marlcov
    torch = torch_cuda
    cfg, shape, p, B, T = BATCH_CASES[name]
    rs = np.random.RandomState(zlib.crc32(name.encode()))
    grids = [tri_valued(rs, 30, 26) if shape == "tri" else bernoulli(rs, shape[0], shape[1], p) for _ in range(B)]
    N = cfg["numrobot"]
    pos = np.stack([draw_positions(rs, g, N) for g in grids])
    env = marlcov.BatchSuperGridEnv(cfg, B, grids=grids, device="cuda", auto_reset=False)
    env.reset(positions=pos)
    refs = []
    for b in range(B):
        np.random.seed(b)
        r = SuperGridRLRef([grids[b]], cfg)
        r.reset(False, None, positions=pos[b])
        refs.append(r)
    st = device_state(env)
    for b in range(B):
        compare(st, b, refs[b], f"{name} reset env {b}")
    for t in range(T):
        digits = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
        quot = rs.choice([0, 0, 0, 1, 2, 3], size=B).astype(np.int32)
        sentinel = rs.rand(B) < 0.05
        codes = digits.copy()
        codes[sentinel, 0] = 255
        (_, _), rew, dn = env.step(torch.from_numpy(codes).cuda(), quot=torch.from_numpy(quot))
        env.check()
        rew, dn = rew.cpu().numpy(), dn.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            if sentinel[b]:
                _, rr, rd = refs[b].step(None)
            else:
                a = int(sum(int(d) * 4 ** i for i, d in enumerate(digits[b]))) + int(quot[b]) * 4 ** N
                _, rr, rd = refs[b].step(a)
            tag = f"{name} step {t} env {b}"
            assert float(rr) == rew[b], (tag, float(rr), rew[b])
            assert bool(rd) == bool(dn[b]), tag
            compare(st, b, refs[b], tag)


def test_super_auto_reset_matches_oracle_reset(torch_cuda):
    import marlcov
    torch = torch_cuda
    cfg = sg_cfg(numrobot=3, senseradius=2, dist_reward=1, use_scanning=1)
    rs = np.random.RandomState(77)
    B, T, cut = 12, 70, 17
    grids = [bernoulli(rs, 18, 22, 0.15) for _ in range(B)]
    pos = np.stack([draw_positions(rs, g, 3) for g in grids])
    env = marlcov.BatchSuperGridEnv(cfg, B, grids=grids, device="cuda", auto_reset=True, maxsteps=cut, seed=5)
    env.reset(positions=pos)
    refs = []
    for b in range(B):
        np.random.seed(b)
        r = SuperGridRLRef([grids[b]], cfg)
        r.reset(False, None, positions=pos[b])
        refs.append(r)
    resets = 0
    for t in range(T):
        digits = rs.randint(0, 4, size=(B, 3)).astype(np.uint8)
        sentinel = rs.rand(B) < 0.03
        codes = digits.copy()
        codes[sentinel, 0] = 255
        (_, _), rew, dn = env.step(torch.from_numpy(codes).cuda())
        env.check()
        rew, dn = rew.cpu().numpy(), dn.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            if sentinel[b]:
                _, rr, rd = refs[b].step(None)
            else:
                _, rr, rd = refs[b].step(int(sum(int(d) * 4 ** i for i, d in enumerate(digits[b]))))
                rd = rd or refs[b]._currstep == cut  # the batch's episode cut (Utils/utils.py:25-28)
            tag = f"auto-reset step {t} env {b}"
            assert float(rr) == rew[b], tag
            assert bool(rd) == bool(dn[b]), tag
            if dn[b]:  # the device reset this env inside the launch
                resets += 1
                refs[b].reset(False, None, positions=st["pos"][b])
                assert (grids[b][st["pos"][b, :, 0], st["pos"][b, :, 1]] >= 0).all(), tag
                assert len({tuple(p) for p in st["pos"][b]}) == 3, tag
            compare(st, b, refs[b], tag)
    assert resets >= B  # every env passed the cut at least once


# ---------------------------------------------------------------------------
# 4. the bench workload at full size
# ---------------------------------------------------------------------------
def oracle_from_device(st, b, cfg):
    g = st["env_grid"][b]
    grid = np.where(st["neg"][g] == 1, -1.0, np.where(st["gpos"][g] == 1, 1.0, 0.0))
    np.random.seed(0)
    ref = SuperGridRLRef([grid], cfg)
    ref._xinds = st["pos"][b, :, 0].astype(int).copy()
    ref._yinds = st["pos"][b, :, 1].astype(int).copy()
    ref._free = 1.0 - st["cov"][b].astype(np.float64)
    ref._observed_obstacles = st["obst"][b].astype(np.float64)
    ref._currstep = int(st["currstep"][b])
    ref._done_thresh = float(st["done_thresh"][b])
    ap = int(st["a_prev"][b])
    ref.a_prev = None if ap < 0 else ap
    return ref


def test_super_bench_workload_full_size(torch_cuda):
    import marlcov
    torch = torch_cuda
    cfg = sg_cfg(numrobot=4, senseradius=2, free_penalty=0.2, dist_reward=1)
    B, W = 4096, 128
    env = marlcov.BatchSuperGridEnv(cfg, B, gen=dict(width=W, length=W, prob_obst=0.1, seed=1000, num_grids=B),
                                    device="cuda", seed=1, auto_reset=True, maxsteps=200)
    env.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for _ in range(40):
        env.step(torch.randint(0, 4, (B, 4), dtype=torch.uint8, device="cuda", generator=g))
    env.check()
    st = device_state(env)
    planes = st["planes"]
    # every env: the uint8 layers are the bitboards and positions
    np.testing.assert_array_equal(planes[:, 4], st["obst"])
    np.testing.assert_array_equal(planes[:, 5], 1 - st["cov"])
    for i in range(4):
        pl = np.zeros((B, W, W), dtype=np.uint8)
        pl[np.arange(B), st["pos"][:, i, 0], st["pos"][:, i, 1]] = 1
        np.testing.assert_array_equal(planes[:, i], pl)
    np.testing.assert_array_equal(st["cov_cnt"], st["cov"].reshape(B, -1).sum(1))
    rs = np.random.RandomState(5)
    sample = rs.choice(B, size=16, replace=False)
    refs = {int(b): oracle_from_device(st, int(b), cfg) for b in sample}
    for b, r in refs.items():
        compare(st, b, r, f"full-size env {b} (rebuilt)")
    for t in range(6):
        digits = rs.randint(0, 4, size=(B, 4)).astype(np.uint8)
        (_, _), rew, dn = env.step(torch.from_numpy(digits).cuda())
        rew, dn = rew.cpu().numpy(), dn.cpu().numpy()
        st = device_state(env)
        for b, r in refs.items():
            _, rr, rd = r.step(int(sum(int(d) * 4 ** i for i, d in enumerate(digits[b]))))
            rd = rd or r._currstep == 200
            assert float(rr) == rew[b] and bool(rd) == bool(dn[b]), (t, b)
            if dn[b]:
                r.reset(False, None, positions=st["pos"][b])
            compare(st, b, r, f"full-size step {t} env {b}")
    env.check()


def test_super_auto_reset_random_grid_pool(torch_cuda):
    """reset_grid_mode="random": every auto-reset lands on the pool grid the
    device drew; the new episode equals an oracle reset there."""
    import marlcov
    torch = torch_cuda
    cfg = sg_cfg(numrobot=2, senseradius=1, dist_reward=1)
    rs = np.random.RandomState(41)
    pool = [bernoulli(rs, 14, 18, 0.2) for _ in range(5)]
    B, cut = 10, 6
    env = marlcov.BatchSuperGridEnv(cfg, B, grids=pool, auto_reset=True, maxsteps=cut, seed=23,
                                    reset_grid_mode="random")
    env.reset()  # every reset draws its grid in this mode, the first one too
    st = device_state(env)
    refs = []
    for b in range(B):
        np.random.seed(b)
        r = SuperGridRLRef([pool[int(st["env_grid"][b])]], cfg)
        r.reset(False, None, positions=st["pos"][b])
        refs.append(r)
        compare(st, b, r, f"random-grid reset env {b}")
    used = set(int(g) for g in st["env_grid"])
    for t in range(36):
        digits = rs.randint(0, 4, size=(B, 2)).astype(np.uint8)
        (_, _), rew, dn = env.step(torch.from_numpy(digits).cuda())
        rew, dn = rew.cpu().numpy(), dn.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            _, rr, rd = refs[b].step(int(digits[b, 0]) + 4 * int(digits[b, 1]))
            rd = rd or refs[b]._currstep == cut
            assert float(rr) == rew[b] and bool(rd) == bool(dn[b]), (t, b)
            if dn[b]:
                g = int(st["env_grid"][b])
                used.add(g)
                a_prev, dt = refs[b].a_prev, refs[b]._done_thresh  # kept across resets
                np.random.seed(0)
                refs[b] = SuperGridRLRef([pool[g]], cfg)
                refs[b].a_prev, refs[b]._done_thresh = a_prev, dt
                refs[b].reset(False, None, positions=st["pos"][b])
            compare(st, b, refs[b], f"random-grid step {t} env {b}")
    assert len(used) >= 4
    env.check()
