"""GPU parity of the compiled-shape kernels the benchmark times.

The env kernel is instantiated per BASELINE workload shape (csrc/
mc_env_kernel.hip select_env: C2, C2D = C2 + dijkstra_input, C4, C5); every
other config runs the generic instantiation.  These tests run each compiled
shape — asserted through mc_kernel_variant — against the oracle
(oracle/cpu_ref.py) every step, including the auto-reset branch inside the
kernel (dec_grid_rl.py:449-531 reached from done() :533-546) and the distance
transform instantiations (csrc/mc_dist.hip dist_kernel_t<16/33/52>).  Device
start cells of every reset are also checked against the host restatement of
the device Philox stream (marlcov.streams.start_cells), and the sharded-batch
property of SURVEY 8(e) (env e's trajectory does not depend on the shard it
runs in) is checked on one GPU with two handles.
"""
import zlib

import numpy as np
import pytest

from gpu_util import compare_env, device_state, oracle_from_device, ref_action
from test_gpu_parity import base_cfg, bern, check_dist_mw, full_obs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def _actions(rs, B, N, sentinel_p=0.05, noop_p=0.06):
    acts = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
    acts[rs.rand(B, N) < noop_p] = rs.choice([4, 9, 254])
    acts[rs.rand(B) < sentinel_p, 0] = 255
    return acts


def run_against_oracle(torch, env, cfg, rs, T, envs, seed, label, dist_check=False, sentinel_p=0.05, on_step=None):
    """Step ``env`` T times with random actions (no-op codes and sentinel rows
    included) and compare the envs in ``envs`` with oracle envs rebuilt from
    the device state after the reset: reward, done, obs (with the float dist
    layer), positions, maps, counters every step; on every done the oracle
    resets at the device-drawn cells, which must equal the host Philox draw.
    Returns the number of auto-resets seen."""
    from marlcov import streams
    B, N = env.num_envs, env.num_agents
    st = device_state(env, envs)
    refs = {b: oracle_from_device(st, b, cfg) for b in envs}
    resets = 0
    for t in range(T):
        acts = _actions(rs, B, N, sentinel_p=sentinel_p)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env, envs)
        for b in envs:
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"{label} t={t} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            assert bool(d) == bool(done_h[b]), tag
            if d:
                resets += 1
                p = st["pos"][b]
                g = int(st["env_grid"][b])
                grid = np.where(st["neg"][g] == 1, -1.0, np.where(st["pos_plane"][g] == 1, 1.0, 0.0))
                want = streams.start_cells(seed, env.env_offset + b, int(st["episode"][b]), grid, N)
                np.testing.assert_array_equal(p, want, err_msg=tag + " start cells vs host Philox")
                o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in p])
                assert int(st["currstep"][b]) == 0, tag
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
        if dist_check:
            check_dist_mw(env, refs, f"{label} t={t}", envs=envs)
        if on_step is not None:
            on_step(t)
    env.check()
    return resets


# (config, unpadded grid side, envs, steps, expected variant tag)
SHAPES = {
    "C2": (base_cfg(numrobot=4, maxsteps=7), 40, 16, 30, "C2"),
    "C2D": (base_cfg(numrobot=4, maxsteps=7, dijkstra_input=1), 40, 16, 30, "C2D"),
    "C4": (base_cfg(numrobot=8, maxsteps=7, allow_even_beams=True, sensor_config={"num_lasers": 360, "range": 20}),
           60, 6, 20, "C4"),
    "C5": (base_cfg(numrobot=16, maxsteps=7, dist_reward=1), 40, 6, 20, "C5"),
}


@pytest.mark.parametrize("name", sorted(SHAPES))
def test_compiled_shape_auto_reset(torch_cuda, name):
    """Every compiled shape with auto_reset and a short episode (maxsteps 7):
    done envs reset inside the step kernel (its reset_env instantiation) and
    the new episode equals the oracle's reset at the device-drawn cells."""
    import marlcov
    torch = torch_cuda
    cfg, side, B, T, tag = SHAPES[name]
    rs = np.random.RandomState(zlib.crc32(name.encode()))
    grids = [bern(rs, side, side, 0.1) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=True, seed=77, env_offset=1000)
    assert f",{tag}>" in env.kernel_variant(), env.kernel_variant()
    env.reset()
    resets = run_against_oracle(torch, env, cfg, rs, T, list(range(B)), 77, name,
                                dist_check=bool(cfg.get("dist_reward")))
    assert resets >= B  # maxsteps=7 over >= 20 steps: every env reset at least twice, less sentinels


@pytest.mark.parametrize("march", ["fan", "rays"])
def test_c4_shape_256_many_envs(torch_cuda, monkeypatch, march):
    """BASELINE configs[3] geometry (8 agents, 256x256, 360 beams, R=20) on
    16 envs x 40 steps through the C4 instantiation, with auto-resets (maxsteps
    13).  358 of the 360 beams share one step pattern over every start and
    march in 64 sectors (fan_march); 270 and 315 degrees march as special
    one-beam sectors from their per-start patterns.  "rays": the ray march
    (MARLCOV_FAN=0)."""
    import marlcov
    torch = torch_cuda
    if march == "rays":
        monkeypatch.setenv("MARLCOV_FAN", "0")
    else:
        monkeypatch.delenv("MARLCOV_FAN", raising=False)
    cfg = base_cfg(numrobot=8, maxsteps=13, allow_even_beams=True, sensor_config={"num_lasers": 360, "range": 20})
    rs = np.random.RandomState(404)
    B = 16
    grids = [bern(rs, 256, 256, 0.1) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=True, seed=5)
    assert ",C4>" in env.kernel_variant(), env.kernel_variant()
    assert ("+fan(64/2)" in env.kernel_variant()) == (march == "fan"), env.kernel_variant()
    env.reset()
    resets = run_against_oracle(torch, env, cfg, rs, 40, list(range(B)), 5, "c4_256", sentinel_p=0.02)
    assert resets >= B


def test_c4_shape_sentinels_and_partial_resets(torch_cuda):
    """The env kernel's non-stepping branch at the C4 compiled shape (four
    waves per env, fan march on): a sentinel row without auto_reset
    (dec_grid_rl.py:104-107: reward 0, done, no state change, obs of the
    current state) and every env left out of a partial mc_reset take it.
    16 envs x 40 steps with sentinel rows at 30 %, plus partial resets with
    an env mask at t = 12 (injected start cells) and t = 27 (device draw), each
    step against the oracle.  Round 3's record: the column-plane scatter of
    this branch raced with another wave's fold / oold stores (wrong obs)."""
    import marlcov
    from marlcov import streams
    torch = torch_cuda
    cfg = base_cfg(numrobot=8, allow_even_beams=True, sensor_config={"num_lasers": 360, "range": 20})
    rs = np.random.RandomState(4040)
    B, N, T = 16, 8, 40
    grids = [bern(rs, 72, 72, 0.1) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=False, seed=9)
    assert ",C4>" in env.kernel_variant() and "+fan(" in env.kernel_variant(), env.kernel_variant()
    env.reset()
    st = device_state(env)
    refs = [oracle_from_device(st, b, cfg) for b in range(B)]
    sentinels = 0
    for t in range(T):
        if t in (12, 27):
            mask = rs.rand(B) < 0.5
            mask[t % B] = True
            mask[(t + 1) % B] = False
            inject = t == 12
            pos = None
            if inject:
                pos = st["pos"].copy()
                for b in np.flatnonzero(mask):
                    g = refs[b]._grid
                    cells = np.argwhere(g >= 0)
                    pick = cells[rs.choice(len(cells), N, replace=False)]
                    pos[b] = pick
            obs = env.reset(env_mask=mask.astype(np.uint8), positions=pos)
            obs_h = full_obs(env, obs, cfg)
            st = device_state(env)
            for b in range(B):
                tag = f"c4 partial reset t={t} env {b}"
                if mask[b]:
                    p = st["pos"][b]
                    if inject:
                        np.testing.assert_array_equal(p, pos[b], err_msg=tag)
                    else:
                        want = streams.start_cells(9, b, int(st["episode"][b]), refs[b]._grid, N)
                        np.testing.assert_array_equal(p, want, err_msg=tag + " start cells vs host Philox")
                    o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in p])
                else:
                    o = refs[b].get_egocentric_observations()
                np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
                compare_env(st, b, refs[b], tag)
        acts = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
        acts[rs.rand(B, N) < 0.06] = 9
        sent = rs.rand(B) < 0.3
        acts[sent, 0] = 255
        sentinels += int(sent.sum())
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"c4 sentinel t={t} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            assert bool(d) == bool(done_h[b]), tag
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
    assert sentinels >= B * T // 5
    env.check()


def test_c5_shape_512_per_step(torch_cuda):
    """BASELINE configs[4] geometry (16 agents, 512x512, dist_reward) on 256
    envs through the C5 instantiation: 8 envs compared with the oracle every
    step from the reset for 30 steps, and every known (max d, witness) of those
    envs checked against a fresh transform every step.  RX = 518 extended rows
    runs the full transform as dist_kernel_t<17> (mc_dist.hip chunk_rows)."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=2000)
    B = 256
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=512, length=512, prob_obst=0.1, seed=1000),
                                   seed=5, auto_reset=True)
    assert ",C5>" in env.kernel_variant(), env.kernel_variant()
    assert env.width + 2 * env.pad == 518
    env.reset()
    assert int(env.get_state(_lib.FIELD_DIST_LISTED).item()) > 0  # reset: M unknown, full transforms
    sample = [0, 17, 64, 101, 150, 200, 233, 255]
    rs = np.random.RandomState(12)
    run_against_oracle(torch, env, cfg, rs, 30, sample, 5, "c5_512", dist_check=True, sentinel_p=0.0)


@pytest.mark.parametrize("dist", [0, 1])
def test_c5_shape_crowded_collisions(torch_cuda, dist):
    """The C5 instantiation's moves (16 robots: moves_par's fixed point over
    the robot order; dist = 0: the generic kernel's serial rounds) where
    robots block each other all the time: 16 robots
    on 12 x 12 grids, every step against the oracle (dec_grid_rl.py:171-204,
    284-310: a robot may enter a cell a lower-index robot vacated this step
    and is blocked by a higher-index robot that has not moved yet).  The
    oracle counts the robot-robot blocks; there must be many, including
    chains (a block that depends on another robot's outcome this step)."""
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=16, maxsteps=25, dist_reward=dist, collision_penalty=2.5)
    rs = np.random.RandomState(1616 + dist)
    B, N, T = 16, 16, 40
    grids = [bern(rs, 12, 12, 0.15) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=True, seed=16)
    # dist_reward: the C5 instantiation (moves_par); without it the generic
    # 16-robot kernel (moves: the serial broadcast rounds)
    want = ",C5>" if dist else "env_kernel<128,1,u32,generic>"
    assert want in env.kernel_variant(), env.kernel_variant()
    env.reset()
    st = device_state(env)
    refs = {b: oracle_from_device(st, b, cfg) for b in range(B)}
    blocks = chains = 0
    for t in range(T):
        acts = rs.randint(0, 4, size=(B, N)).astype(np.uint8)
        acts[rs.rand(B, N) < 0.05] = 7
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env)
        for b in range(B):
            ref = refs[b]
            x0, y0 = ref._xinds.copy(), ref._yinds.copy()
            start = {(int(x0[i]), int(y0[i])): i for i in range(N)}
            o, r, d = ref.step(ref_action(acts[b]))
            for i in range(N):
                a = int(acts[b, i])
                if a > 3 or (ref._xinds[i], ref._yinds[i]) != (x0[i], y0[i]):
                    continue
                tx, ty = x0[i] + (a == 0) - (a == 2), y0[i] + (a == 1) - (a == 3)
                if ref._grid[tx, ty] >= 0:  # free target: another robot blocked it
                    blocks += 1
                    j = start.get((int(tx), int(ty)))
                    chains += int(j is not None and j < i)  # j < i stayed: its own outcome decided i's
            tag = f"c5 crowded t={t} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            assert bool(d) == bool(done_h[b]), tag
            if d:
                o, _ = ref.reset(False, None, positions=[tuple(q) for q in st["pos"][b]])
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, ref, tag)
    assert blocks > 200 and chains > 20, (blocks, chains)
    env.check()


def test_c5_top_cell_cache_is_exact(torch_cuda, monkeypatch):
    """The dist_reward top-cell cache (mc_dist.hip: the cells with d >= M -
    kDistT, T = 20, and the box of cells covered since) against the full
    transform (MARLCOV_DIST_CACHE=0): 64 C5 envs x 120 steps of the same
    device actions, auto-resets every 45 steps, give bit-identical obs,
    rewards, dones and (max d, witness distance) -- max d is exact whichever
    path made it.  The cache handle must have served listed maps
    (MC_FIELD_DIST_CACHED); the oracle checks of the cache are
    test_c5_cache_steady_state_matches_oracle and test_c5_shape_512_per_step."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=45)
    B = 64
    outs = []
    served = {}
    for cache in ("1", "0"):
        monkeypatch.setenv("MARLCOV_DIST_CACHE", cache)
        env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=512, length=512, prob_obst=0.1, seed=1000),
                                       seed=5, auto_reset=True)
        assert ",C5>" in env.kernel_variant(), env.kernel_variant()
        env.reset()
        acc = []
        served[cache] = 0
        for t in range(120):
            obs, rew, done = env.step(env.random_actions(777, t))
            mw = env.get_state(_lib.FIELD_DIST_MW)[..., 0]
            served[cache] += int(env.get_state(_lib.FIELD_DIST_CACHED).item())
            acc.append((obs.clone(), env.dist_obs.clone(), rew.clone(), done.clone(), mw.clone()))
        outs.append(acc)
    assert served["1"] > 0 and served["0"] == 0, served
    for t, (a, b) in enumerate(zip(*outs)):
        for x, y, name in zip(a[:4], b[:4], ("obs", "dist_obs", "reward", "done")):
            assert torch.equal(x, y), f"step {t}: {name}"
        known = (a[4] >= 0) & (b[4] >= 0)  # max d of the maps both handles know
        assert torch.equal(a[4][known], b[4][known]), f"step {t}: max_d"


def test_c5_unsplit_transform_is_identical(torch_cuda, monkeypatch):
    """MARLCOV_DIST_SPLIT=0 (each listed map tried and, if needed, transformed
    whole by one workgroup: dist_kernel_t mode 1, reading the env kernel's
    sharded work list directly) against the default path (cache tries in
    dist_fast_kernel, full transforms split over parts): 64 C5 envs x 80
    steps of the same device actions give bit-identical obs, distance layers,
    rewards and dones (dec_grid_rl.py:222-223,239-240,260-282)."""
    import marlcov
    torch = torch_cuda
    cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=50)
    outs = []
    for split in ("1", "0"):
        monkeypatch.setenv("MARLCOV_DIST_SPLIT", split)
        env = marlcov.BatchCoverageEnv(cfg, 64, gen=dict(width=512, length=512, prob_obst=0.1, seed=1001),
                                       seed=9, auto_reset=True)
        assert ",C5>" in env.kernel_variant(), env.kernel_variant()
        env.reset()
        acc = []
        for t in range(80):
            obs, rew, done = env.step(env.random_actions(31, t))
            acc.append((obs.clone(), env.dist_obs.clone(), rew.clone(), done.clone()))
        outs.append(acc)
        del env
    for t, (a, b) in enumerate(zip(*outs)):
        for x, y, name in zip(a, b, ("obs", "dist_obs", "reward", "done")):
            assert torch.equal(x, y), f"step {t}: {name}"


def test_c5_cache_steady_state_matches_oracle(torch_cuda, monkeypatch):
    """The top-cell cache where the C5 bench line gets its speed: 256 C5 envs
    (16 agents, 512 x 512, dist_reward, 2000-step episodes) run 600 device
    random-action steps; 6 envs are then rebuilt in the oracle from device
    state (oracle_from_device) and 25 more steps are compared with it every
    step -- reward (float32 distance terms), done, obs with the float distance
    layer, maps, counters -- and every known (max d, witness) against a fresh
    transform (check_dist_mw; dec_grid_rl.py:222-223,239-240,260-282).  Most
    of the maps those steps list for the full transform must be served by the
    cache fast path (MC_FIELD_DIST_CACHED / MC_FIELD_DIST_LISTED)."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    monkeypatch.setenv("MARLCOV_DIST_CACHE", "1")
    cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=2000)
    B = 256
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=512, length=512, prob_obst=0.1, seed=1000),
                                   seed=5, auto_reset=True)
    assert ",C5>" in env.kernel_variant(), env.kernel_variant()
    env.reset()
    for t in range(600):
        env.step(env.random_actions(4242, t))
    env.check()
    sample = [3, 40, 97, 128, 190, 251]
    st = device_state(env, sample)
    assert all(int(st["currstep"][b]) == 600 for b in sample)
    refs = {b: oracle_from_device(st, b, cfg) for b in sample}
    listed = cached = 0
    rs = np.random.RandomState(600)
    for t in range(25):
        acts = rs.randint(0, 4, size=(B, 16)).astype(np.uint8)
        obs, rew, done = env.step(torch.from_numpy(acts).to(env.device))
        listed += int(env.get_state(_lib.FIELD_DIST_LISTED).item())
        cached += int(env.get_state(_lib.FIELD_DIST_CACHED).item())
        obs_h, rew_h, done_h = full_obs(env, obs, cfg), rew.cpu().numpy(), done.cpu().numpy()
        st = device_state(env, sample)
        for b in sample:
            o, r, d = refs[b].step(ref_action(acts[b]))
            tag = f"c5 steady t={601 + t} env {b}"
            assert float(r) == rew_h[b], (tag, float(r), rew_h[b])
            assert bool(d) == bool(done_h[b]), tag
            if d:  # covered: the device reset the env in the same launch
                o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in st["pos"][b]])
            np.testing.assert_array_equal(obs_h[b], o, err_msg=tag + " obs")
            compare_env(st, b, refs[b], tag)
        check_dist_mw(env, refs, f"c5 steady t={601 + t}", envs=sample)
    assert listed > 0 and 2 * cached > listed, (listed, cached)
    env.check()


@pytest.mark.parametrize("rows,rx", [(600, 606), (538, 544)], ids=["rx606_kcl26", "rx544_kcl17_full"])
def test_dist_kernel_long_maps(torch_cuda, rows, rx):
    """Extended maps of 545..832 rows run the transform as dist_kernel_t<26>
    (a 600 x 40 grid, RX = 606); RX = 544 fills the 32 chunks of 17 rows of
    dist_kernel_t<17> exactly (no padding row).  dist_reward, per step
    against the oracle."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    cfg = base_cfg(numrobot=2, dist_reward=1, sensor_config={"num_lasers": 9, "range": 4})
    rs = np.random.RandomState(rows)
    B = 4
    grids = [bern(rs, rows, 40, 0.1) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(cfg, B, grids=grids, auto_reset=False)
    assert env.width + 2 * env.pad == rx
    env.reset()
    assert int(env.get_state(_lib.FIELD_DIST_LISTED).item()) > 0
    run_against_oracle(torch, env, cfg, rs, 20, list(range(B)), 0, f"dist{rx}", dist_check=True, sentinel_p=0.0)


# ---------------------------------------------------------------------------
# every device stream keyed by the global env id
# ---------------------------------------------------------------------------
def test_shards_reproduce_one_batch(torch_cuda):
    """Two handles holding envs [0, B) and [B, 2B) of a global batch (env
    offsets 0 and B) reproduce one 2B handle bit for bit over 50 auto-reset
    steps at the C2 shape: grids (mc_generate_grids), start cells, actions
    (mc_random_actions), obs, rewards, dones and maps.  The grids, the first
    start cells and the actions also equal the host restatement of the
    streams (marlcov.streams)."""
    import marlcov
    from marlcov import _lib, streams
    torch = torch_cuda
    cfg = base_cfg(numrobot=4, maxsteps=9)
    B, S = 64, 50
    gen = dict(width=64, length=64, prob_obst=0.1, seed=1000)

    def make(n, off):
        e = marlcov.BatchCoverageEnv(cfg, n, gen=dict(gen, num_grids=n), seed=1, auto_reset=True,
                                     env_offset=off)
        e.reset()
        return e

    whole, lo, hi = make(2 * B, 0), make(B, 0), make(B, B)
    assert ",C2>" in whole.kernel_variant()
    # host restatement of the grid pool and the first start cells
    st = device_state(whole, [0, 5, B + 3])
    for b in (0, 5, B + 3):
        want = streams.generated_grid(1000, 0.1, 66, 66, b)
        got = np.where(st["neg"][b] == 1, -1.0, 1.0)
        np.testing.assert_array_equal(got, want, err_msg=f"grid {b}")
        np.testing.assert_array_equal(st["pos"][b], streams.start_cells(1, b, 1, want, 4), err_msg=f"cells {b}")
    for t in range(S):
        a_w = whole.random_actions(12345, t)
        a_l, a_h = lo.random_actions(12345, t), hi.random_actions(12345, t)
        assert torch.equal(a_w, torch.cat([a_l, a_h]))
        if t in (0, 17):
            np.testing.assert_array_equal(a_w.cpu().numpy(), streams.random_actions(12345, range(2 * B), t, 4))
        ow, rw, dw = whole.step(a_w)
        ol, rl, dl = lo.step(a_l)
        oh, rh, dh = hi.step(a_h)
        assert torch.equal(ow, torch.cat([ol, oh])), t
        assert torch.equal(rw, torch.cat([rl, rh])) and torch.equal(dw, torch.cat([dl, dh])), t
    for f in (_lib.FIELD_POS, _lib.FIELD_FREE, _lib.FIELD_OBST, _lib.FIELD_VISITED, _lib.FIELD_EPISODE,
              _lib.FIELD_FREE_COUNT, _lib.FIELD_CURRSTEP):
        assert torch.equal(whole.get_state(f), torch.cat([lo.get_state(f), hi.get_state(f)])), f
    assert int(whole.get_state(_lib.FIELD_EPISODE).min()) >= 5  # maxsteps 9 over 50 steps
    for e in (whole, lo, hi):
        e.check()


@pytest.mark.parametrize("B", [64, 8])
def test_c5_split_maps_across_auto_reset_match_oracle(torch_cuda, B):
    """C5 geometry (16 agents, 512 x 512, dist_reward) across the first
    auto-reset: B envs, maxsteps 50, two envs tracked by the oracle from the
    reset through step 55 (reward with the float32 distance terms, the float
    distance obs layer, maps; every known (max d, witness) against a fresh
    transform).  The steps before the reset split their few full transforms
    over parts (<= 256 maps on the full list); step 50 resets every map at
    once (all caches dropped, B x 16 maps listed).  B = 64: 1,024 maps, one
    workgroup each; B = 8: 128 maps split over parts with no cache bound
    (theta0 = 0: the part lists, and their merge).
    dec_grid_rl.py:222-223,239-240,260-282,449-531."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=50)
    env = marlcov.BatchCoverageEnv(cfg, B, gen=dict(width=512, length=512, prob_obst=0.1, seed=1001),
                                   seed=9, auto_reset=True)
    assert ",C5>" in env.kernel_variant(), env.kernel_variant()
    env.reset()
    tot = [env.get_state(_lib.FIELD_DIST_TOTALS).cpu().tolist()]
    fulls = []  # maps fully transformed per step (MC_FIELD_DIST_TOTALS deltas)

    def on_step(t):
        tot.append(env.get_state(_lib.FIELD_DIST_TOTALS).cpu().tolist())
        fulls.append(tot[-1][2] - tot[-2][2])
    resets = run_against_oracle(torch, env, cfg, np.random.RandomState(55), 55, [1, B - 2], 9, f"c5 reset B={B}",
                                dist_check=True, sentinel_p=0.0, on_step=on_step)
    assert resets == 2  # both tracked envs reset at step 50, once
    assert int(env.get_state(_lib.FIELD_CURRSTEP).max()) == 5
    msg = " ".join(map(str, fulls))
    assert fulls[49] == 16 * B, msg  # step 50: the mass reset sends every map to the full transform
    if B == 64:
        assert any(0 < f <= 256 for f in fulls[:49]), msg  # split steps before it
    else:
        assert all(f <= 256 for f in fulls), msg  # every full transform split, the reset's too


def test_dist_totals_bookkeeping(torch_cuda, monkeypatch):
    """MC_FIELD_DIST_TOTALS (the counters bench.py prices C5's design bytes
    with): over K steps, launches == K, listed == served + full, and listed
    equals the sum of the per-step MC_FIELD_DIST_LISTED values -- with the
    split path (cache tries + split transforms) and with MARLCOV_DIST_SPLIT=0
    (one workgroup per listed map); both paths count the same maps."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=2000)
    res = {}
    for split in ("1", "0"):
        monkeypatch.setenv("MARLCOV_DIST_SPLIT", split)
        env = marlcov.BatchCoverageEnv(cfg, 32, gen=dict(width=512, length=512, prob_obst=0.1, seed=77),
                                       seed=4, auto_reset=True)
        env.reset()
        for t in range(40):  # past the early phase's densest lists
            env.step(env.random_actions(8, t))
        t0 = env.get_state(_lib.FIELD_DIST_TOTALS).cpu().tolist()
        listed = served = 0
        K = 30
        for t in range(40, 40 + K):
            env.step(env.random_actions(8, t))
            listed += int(env.get_state(_lib.FIELD_DIST_LISTED).item())
            served += int(env.get_state(_lib.FIELD_DIST_CACHED).item())
        t1 = env.get_state(_lib.FIELD_DIST_TOTALS).cpu().tolist()
        d = [b - a for a, b in zip(t0, t1)]
        assert d[3] == K, (split, d)
        assert d[0] == d[1] + d[2], (split, d)
        assert d[0] == listed and d[1] == served, (split, d, listed, served)
        assert d[0] > 0, d
        res[split] = d[0]
        del env
    assert res["1"] == res["0"], res  # the same maps listed either way
