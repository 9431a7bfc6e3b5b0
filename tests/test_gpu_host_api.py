"""GPU tests of the host-side API edges: grid pools given as lists of lists,
sensors shared between envs, beam tables that outgrow the LDS budget."""
import gc
import weakref

import numpy as np
import pytest

from oracle.cpu_ref import DecGridRLRef

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def cfg(**kw):
    c = dict(numrobot=2, maxsteps=1000, collision_penalty=5, done_thresh=1, done_incr=0,
             terminal_reward=30, dist_reward=0, train_maxsteps=1000, test_maxsteps=1000,
             egoradius=2, mini_map_rad=0, comm_radius=0, allow_comm=0, map_sharing=0,
             single_square_tool=0, dijkstra_input=0, sensor_type="lidar",
             sensor_config={"num_lasers": 9, "range": 4})
    c.update(kw)
    return c


def test_list_grids_many_resets_match_oracle(torch_cuda):
    """The reference np.pads whatever the train list holds, so lists of lists
    work there (dec_grid_rl.py:466-472): every reset on them must too, across
    grid shapes and with a list entry replaced between episodes."""
    import marlcov
    rs = np.random.RandomState(7)
    mk = lambda w, l: np.where(rs.rand(w, l) < 0.15, -1.0, 1.0).tolist()  # noqa: E731
    train = [mk(12, 12), mk(12, 12), mk(10, 14)]
    c = cfg()
    np.random.seed(3)
    env = marlcov.DecGridRL(train, c)
    np.random.seed(3)
    ref = DecGridRLRef(train, c)
    for ep in range(8):
        if ep in (3, 5, 6):
            train[1] = mk(12, 12)  # a new object of an existing shape
        seed = 100 + ep
        np.random.seed(seed)
        o, g = env.reset(False, None)
        np.random.seed(seed)
        ro, rg = ref.reset(False, None)
        np.testing.assert_array_equal(g, rg)
        np.testing.assert_array_equal(o, ro)
        for t in range(6):
            a = int(rs.randint(0, 16))
            o, r, d = env.step(a)
            ro, rr, rd = ref.step(a)
            tag = f"ep {ep} t {t}"
            assert float(r) == float(rr), tag
            assert bool(d) == bool(rd), tag
            np.testing.assert_array_equal(o, ro, err_msg=tag)
    # replaced entries leave the pool at the next rebuild: it never grows past
    # the lists' two 12x12 grids
    pool = env._envs[(14, 14)][1]
    assert len(pool) == 2 and pool[0] is train[0]
    assert sum(v[0] == (14, 14) for v in env._pool_index.values()) == 2


def test_shared_sensor_does_not_keep_envs_alive(torch_cuda):
    import marlcov
    c = cfg()
    from marlcov.sensors import make_sensor
    sensor = make_sensor(c)
    grid = np.ones((16, 16))
    e1 = marlcov.BatchCoverageEnv(c, 2, grids=[grid], sensor=sensor)
    e2 = marlcov.BatchCoverageEnv(c, 2, grids=[grid], sensor=sensor)
    w1 = weakref.ref(e1)
    del e1
    gc.collect()
    assert w1() is None, "the sensor kept a device env alive"
    e2.close()
    sensor.set_thetalist(np.linspace(0, 2 * np.pi, 11, endpoint=False))  # no listener left to fail
    assert sensor._listeners == []


def test_beam_table_over_lds_budget_is_rejected(torch_cuda):
    """A beam count that no longer fits the per-env LDS window mc_create
    checked is refused when the table is set, with a clear error."""
    import marlcov
    env = marlcov.BatchCoverageEnv(cfg(), 1, grids=[np.ones((20, 20))])
    other = marlcov.BatchCoverageEnv(cfg(), 1, grids=[np.ones((20, 20))], sensor=env.sensor)
    n0 = env.sensor._num_lasers
    with pytest.raises(Exception, match="LDS"):  # 16 B per beam: 4500 beams > 64 KiB
        env.sensor.set_thetalist(np.linspace(0, 2 * np.pi, 4500, endpoint=False))
    # the old table is still the one in effect everywhere
    assert env.sensor._num_lasers == n0 and len(env.sensor._thetalist) == n0
    assert env._cfg.num_beams == n0 and other._cfg.num_beams == n0
    for e in (env, other):
        e.reset(positions=np.array([[[5, 5], [7, 9]]], dtype=np.int32))
        e.check()
    # the shared sensor's two envs see the same cells after the rejection
    assert env.obs.cpu().numpy().tobytes() == other.obs.cpu().numpy().tobytes()
    assert len(env.sensor._listeners) == 2


def test_rollout_matches_steps_and_oracle(torch_cuda):
    """mc_step_many (BatchCoverageEnv.rollout): K steps in one C-ABI call give
    step k's obs / reward / done exactly as K mc_step calls do, and as the
    oracle's K steps (dec_grid_rl.py:91-169), auto-resets included; the env
    state after the rollout equals the stepped env's."""
    import marlcov
    from marlcov import _lib
    from gpu_util import compare_env, device_state, oracle_from_device, ref_action
    torch = torch_cuda
    c = cfg(numrobot=3, maxsteps=9)
    rs = np.random.RandomState(99)
    B, K = 8, 24
    grids = [np.where(rs.rand(20, 20) < 0.15, -1.0, 1.0) for _ in range(B)]
    envs = [marlcov.BatchCoverageEnv(c, B, grids=grids, auto_reset=True, seed=3) for _ in range(2)]
    for e in envs:
        e.reset()
    acts = rs.randint(0, 4, size=(K, B, 3)).astype(np.uint8)
    acts[rs.rand(K, B) < 0.1, 0] = 255
    st = device_state(envs[0])
    refs = [oracle_from_device(st, b, c) for b in range(B)]
    obs_r, rew_r, done_r = envs[0].rollout(torch.from_numpy(acts).to(envs[0].device))
    for k in range(K):
        o, r, d = envs[1].step(torch.from_numpy(acts[k]).to(envs[1].device))
        assert torch.equal(o, obs_r[k]) and torch.equal(r, rew_r[k]) and torch.equal(d, done_r[k]), k
        for b in range(B):
            oo, rr, dd = refs[b].step(ref_action(acts[k, b]))
            assert float(rr) == float(rew_r[k, b]) and bool(dd) == bool(done_r[k, b]), (k, b)
            if dd:
                p = envs[1].get_state(_lib.FIELD_POS).cpu().numpy()[b]  # the stepped env, after step k
                oo, _ = refs[b].reset(False, None, positions=[tuple(q) for q in p])
            np.testing.assert_array_equal(obs_r[k, b].cpu().numpy(), oo, err_msg=f"k={k} b={b}")
    st0, st1 = device_state(envs[0]), device_state(envs[1])
    for b in range(B):
        compare_env(st0, b, refs[b], f"rollout end env {b}")
        compare_env(st1, b, refs[b], f"stepped end env {b}")
    assert int(done_r.sum()) >= B  # maxsteps 9 over 24 steps
    for e in envs:
        e.check()


def test_rollout_per_step_adjacency_and_float_layers(torch_cuda):
    """rollout on a comm-graph config returns every step's adjacency
    (dec_grid_rl.py:374-391 after each step's moves), equal to K step calls;
    a dist_reward config (one registered float obs buffer) is refused rather
    than silently keeping only the last step's float layer; mc_step_many
    rejects a reward stride that is not a multiple of 8."""
    import marlcov
    torch = torch_cuda
    c = cfg(numrobot=4, maxsteps=7, comm_radius=5, allow_comm=1)
    rs = np.random.RandomState(5)
    B, K = 6, 15
    grids = [np.where(rs.rand(18, 18) < 0.1, -1.0, 1.0) for _ in range(B)]
    envs = [marlcov.BatchCoverageEnv(c, B, grids=grids, auto_reset=True, seed=4, want_adjacency=True)
            for _ in range(2)]
    for e in envs:
        e.reset()
    acts = torch.from_numpy(rs.randint(0, 4, size=(K, B, 4)).astype(np.uint8)).to(envs[0].device)
    (obs_r, adj_r), rew_r, done_r = envs[0].rollout(acts)
    assert tuple(adj_r.shape) == (K, B, 4, 4)
    changed = 0
    for k in range(K):
        (o, a), r, d = envs[1].step(acts[k])
        assert torch.equal(o, obs_r[k]) and torch.equal(a, adj_r[k]), k
        assert torch.equal(r, rew_r[k]) and torch.equal(d, done_r[k]), k
        changed += int(k > 0 and not torch.equal(adj_r[k], adj_r[k - 1]))
    assert changed > 0  # the graph moves with the robots: per-step values, not the last one repeated
    assert torch.equal(envs[0].adj, adj_r[-1])
    dc = cfg(numrobot=2, dist_reward=1, sensor_config={"num_lasers": 9, "range": 4})
    de = marlcov.BatchCoverageEnv(dc, 2, grids=grids[:2], auto_reset=True)
    de.reset()
    with pytest.raises(ValueError, match="float obs"):
        de.rollout(torch.zeros((3, 2, 2), dtype=torch.uint8, device=de.device))
    e = envs[1]
    rc = e.lib.mc_step_many(e._h, acts.data_ptr(), B * 4, 1, e.reward.data_ptr(), 4, e.done.data_ptr(), 0,
                            e.obs.data_ptr(), 0, None, 0, e._stream())
    assert rc != 0 and b"multiple of 8" in e.lib.mc_last_error()
    for x in envs + [de]:
        x.check()
