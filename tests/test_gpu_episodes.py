"""GPU: the batched episode driver (marlcov.episodes)
against the oracle running the reference's generate_episode loop
(Utils/utils.py:6-44) on the same actions and the device-drawn start cells:
per-episode total reward, length and final percent_covered() bit-exact."""
import numpy as np
import pytest

from gpu_util import device_state, oracle_from_device, ref_action

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def cfg(**kw):
    c = dict(numrobot=3, maxsteps=1000, collision_penalty=5, done_thresh=0.35, done_incr=0.1,
             terminal_reward=30, dist_reward=0, train_maxsteps=1000, test_maxsteps=14, egoradius=2,
             mini_map_rad=0, comm_radius=0, allow_comm=0, map_sharing=0, single_square_tool=0,
             dijkstra_input=0, sensor_type="lidar", sensor_config={"num_lasers": 11, "range": 4})
    c.update(kw)
    return c


@pytest.mark.parametrize("dist", [0, 1])
def test_generate_episodes_matches_oracle_loop(torch_cuda, dist):
    import marlcov
    from marlcov.episodes import episode_config, generate_episodes, random_policy
    torch = torch_cuda
    c = episode_config(cfg(dist_reward=dist), testing=True)
    assert c["maxsteps"] == 14
    rs = np.random.RandomState(11 + dist)
    B, E = 10, 4
    grids = [rs.choice([1.0, -1.0], size=(16, 16), p=[0.85, 0.15]) for _ in range(B)]
    env = marlcov.BatchCoverageEnv(c, B, grids=grids, auto_reset=True, seed=9)
    env.reset()
    st = device_state(env)
    refs = [oracle_from_device(st, b, c) for b in range(B)]
    episodes = [[] for _ in range(B)]
    acc = np.zeros(B)
    base = random_policy(env, seed=4)
    gsent = np.random.RandomState(5)

    def policy(obs):
        a = base(obs)
        a[torch.from_numpy(gsent.rand(B) < 0.04).to(env.device), 0] = 255  # sentinel ends an episode
        return a

    def on_step(t, actions, reward, done):
        acts = actions.cpu().numpy()
        rew, dn = reward.cpu().numpy(), done.cpu().numpy()
        s = device_state(env)
        for b in range(B):
            _, r, d = refs[b].step(ref_action(acts[b]))
            assert float(r) == rew[b] and bool(d) == bool(dn[b]), (t, b)
            acc[b] += r
            if d:
                episodes[b].append((acc[b], refs[b]._currstep, refs[b].percent_covered()))
                acc[b] = 0.0
                refs[b].reset(False, None, positions=[tuple(q) for q in s["pos"][b]])

    out = generate_episodes(env, policy, E, max_steps=2000, on_step=on_step)
    for b in range(B):
        assert len(episodes[b]) >= E
        for k in range(E):
            r, n, pc = episodes[b][k]
            assert out["reward"][b, k] == r, (b, k, out["reward"][b, k], r)
            assert out["length"][b, k] == n, (b, k)
            assert out["percent_covered"][b, k] == pc, (b, k)
    assert (out["length"] <= 14).all() and (out["length"] >= 0).all()


def test_batched_test_RLalg_statistics(torch_cuda):
    import marlcov
    from marlcov.episodes import random_policy, test_RLalg
    train, test = marlcov.gridload(None)  # the reference's hand-made 15x15 grids
    c = cfg(numrobot=1, test_maxsteps=30, done_thresh=1, done_incr=0, sensor_type="square_sensor",
            sensor_config={"range": 1})
    rewards, avg = test_RLalg(c, test, lambda env: random_policy(env, seed=1), episodes=8, envs_per_grid=4)
    assert len(rewards) == 8 * len(test)
    assert 0.0 < avg <= 100.0
    # a 30-step episode of 1 robot with a 3x3 sensor cannot cover a 15x15 grid
    assert all(-5 * 30 <= r <= 9 * 30 for r in rewards)


def test_generate_episodes_super_matches_oracle_loop(torch_cuda):
    """The same driver over BatchSuperGridEnv (grid_rl_main.py can run either
    env): per-episode return, length and percent_covered() vs the oracle."""
    import marlcov
    from marlcov import _lib
    from marlcov.episodes import generate_episodes, random_policy
    from marlcov.super_env import decode_super_action  # noqa: F401  (API surface)
    from oracle.super_ref import SuperGridRLRef
    torch = torch_cuda
    c = dict(numrobot=3, train_maxsteps=1000, test_maxsteps=1000, collision_penalty=5, senseradius=1,
             free_penalty=0.2, done_thresh=0.5, done_incr=0.1, terminal_reward=30, dist_reward=1,
             use_scanning=1)
    rs = np.random.RandomState(21)
    B, E, cut = 8, 3, 16
    grids = [rs.choice([1.0, -1.0], size=(12, 14), p=[0.85, 0.15]) for _ in range(B)]
    env = marlcov.BatchSuperGridEnv(c, B, grids=grids, auto_reset=True, maxsteps=cut, seed=3)
    env.reset()
    pos = env.get_state(_lib.SG_FIELD_POS).cpu().numpy()
    refs = []
    for b in range(B):
        np.random.seed(b)
        r = SuperGridRLRef([grids[b]], c)
        r.reset(False, None, positions=pos[b])
        refs.append(r)
    episodes = [[] for _ in range(B)]
    acc = np.zeros(B)
    base = random_policy(env, seed=8)

    def on_step(t, actions, reward, done):
        acts = actions.cpu().numpy()
        rew, dn = reward.cpu().numpy(), done.cpu().numpy()
        p = env.get_state(_lib.SG_FIELD_POS).cpu().numpy()
        for b in range(B):
            _, r, d = refs[b].step(int(sum(int(x) * 4 ** i for i, x in enumerate(acts[b]))))
            d = d or refs[b]._currstep == cut
            assert float(r) == rew[b] and bool(d) == bool(dn[b]), (t, b)
            acc[b] += r
            if d:
                episodes[b].append((acc[b], refs[b]._currstep, refs[b].percent_covered()))
                acc[b] = 0.0
                refs[b].reset(False, None, positions=p[b])

    out = generate_episodes(env, base, E, max_steps=1000, on_step=on_step)
    for b in range(B):
        for k in range(E):
            r, n, pc = episodes[b][k]
            assert out["reward"][b, k] == r and out["length"][b, k] == n, (b, k)
            assert out["percent_covered"][b, k] == pc, (b, k)
