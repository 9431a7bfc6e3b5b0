"""Batched episode driver: the reference's ``Utils/utils.py`` loop
(``generate_episode`` :6-44, ``test_RLalg`` :111-149) for B envs at once.

Every env of a ``BatchCoverageEnv`` (``auto_reset=True``) runs its own
sequence of episodes; the per-episode total reward, length and final
``percent_covered()`` (what ``test_RLalg`` averages, :141) are collected on
the device from the kernel's episode record (``MC_FIELD_EP_PC`` /
``MC_FIELD_EP_LEN``, written before an auto-reset clears the counters).  The
host only launches steps and checks for completion every few steps.

Episode cut: ``generate_episode`` ends an episode when ``_currstep`` reaches
``_test_maxsteps`` / ``_train_maxsteps`` (:25-28), and ``DecGridRL.done()``
at ``maxsteps`` (dec_grid_rl.py:544); ``episode_config`` folds both into the
env's ``maxsteps`` (the smaller one ends the episode first, with the same
reward), so the kernel's done is the loop's done.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def episode_config(env_config, testing):
    """env_config whose ``maxsteps`` is the episode cut of utils.py:25-28."""
    c = dict(env_config)
    cut = c["test_maxsteps"] if testing else c["train_maxsteps"]
    c["maxsteps"] = min(int(c["maxsteps"]), int(cut))
    return c


def random_policy(env, seed=0):
    """Uniform per-agent actions in {0..3} from a seeded device generator
    (the ``Discrete.sample`` of Action_Spaces/discrete.py, batched)."""
    torch = env._torch
    g = torch.Generator(device=env.device)
    g.manual_seed(seed)
    shape = (env.num_envs, env.num_agents)

    def pi(_obs):
        return torch.randint(0, 4, shape, dtype=torch.uint8, device=env.device, generator=g)
    return pi


def _record_fields(env):
    """(get_state function, episode-record fields) of a batch env type."""
    if hasattr(env, "planes"):  # BatchSuperGridEnv
        return env.lib.mc_sg_get_state, (_lib.SG_FIELD_EP_PC, _lib.SG_FIELD_EP_LEN)
    return env.lib.mc_get_state, (_lib.FIELD_EP_PC, _lib.FIELD_EP_LEN)


def generate_episodes(env, policy, episodes_per_env, max_steps=None, on_step=None, check_every=16):
    """Run every env of ``env`` (a BatchCoverageEnv or BatchSuperGridEnv with
    auto_reset) until it
    finished ``episodes_per_env`` episodes.  ``policy(obs) -> uint8 [B, N]``
    device actions (255 in agent 0 = the sentinel, which ends the episode as
    in generate_episode).  ``on_step(t, actions, reward, done)`` is called
    after every step (tests use it to follow the device).

    Returns a dict of numpy arrays [B, episodes_per_env]: ``reward`` (the
    float64 sum of the episode's step rewards, generate_episode's
    total_reward), ``length`` (steps) and ``percent_covered`` (at the end).
    Envs that finish early keep running (a batch steps every env) but record
    nothing more."""
    if not env._cfg.auto_reset:
        raise ValueError("generate_episodes needs a batch env with auto_reset=True")
    torch = env._torch
    B, E = env.num_envs, int(episodes_per_env)
    dev = env.device
    rec_ret = torch.zeros((B, E), dtype=torch.float64, device=dev)
    rec_len = torch.zeros((B, E), dtype=torch.int32, device=dev)
    rec_pc = torch.zeros((B, E), dtype=torch.float64, device=dev)
    count = torch.zeros(B, dtype=torch.int64, device=dev)
    ret = torch.zeros(B, dtype=torch.float64, device=dev)
    ep_pc = torch.empty(B, dtype=torch.float64, device=dev)
    ep_len = torch.empty(B, dtype=torch.int32, device=dev)
    rows = torch.arange(B, device=dev)
    get_state, (f_pc, f_len) = _record_fields(env)
    if hasattr(env, "planes"):
        obs = (env.planes, env.dist)
    else:
        obs = env.obs if env.adj is None else (env.obs, env.adj)
    t = 0
    while True:
        actions = policy(obs)
        obs, reward, done = env.step(actions)
        ret += reward
        for field, buf in ((f_pc, ep_pc), (f_len, ep_len)):
            _lib.check(get_state(env._h, field, buf.data_ptr(), buf.numel() * buf.element_size(),
                                 env._stream()), "get_state")
        d = done.bool()
        take = d & (count < E)
        idx = count.clamp(max=E - 1)
        rec_ret[rows, idx] = torch.where(take, ret, rec_ret[rows, idx])
        rec_len[rows, idx] = torch.where(take, ep_len, rec_len[rows, idx])
        rec_pc[rows, idx] = torch.where(take, ep_pc, rec_pc[rows, idx])
        count += take
        ret.masked_fill_(d, 0.0)
        t += 1
        if on_step is not None:
            on_step(t, actions, reward, done)
        if t % check_every == 0 or on_step is not None:
            if bool((count >= E).all()):
                break
        if max_steps is not None and t >= max_steps:
            raise RuntimeError(f"episodes not finished after {max_steps} steps")
    env.check()
    return {"reward": rec_ret.cpu().numpy(), "length": rec_len.cpu().numpy(),
            "percent_covered": rec_pc.cpu().numpy(), "steps": t}


def test_RLalg(env_config, test_grids, policy_factory, episodes=100, envs_per_grid=None, device="cuda",
               seed=0, **env_kw):
    """Batched ``test_RLalg`` (utils.py:111-149): ``episodes`` test episodes
    on every grid of ``test_grids`` (unpadded), run in parallel —
    ``envs_per_grid`` envs per grid (default: ``episodes``), each running
    ``episodes / envs_per_grid`` of them.  ``policy_factory(env)`` returns the
    batched policy.  Returns ``(test_rewardlis, average_percent_covered)``
    like the reference: the per-episode total rewards (grid-major) and the
    mean percent covered x 100.  Start cells come from the device Philox
    stream (same distribution as the reference's NumPy draw, not its bits)."""
    from .batch_env import BatchCoverageEnv

    k = int(envs_per_grid or episodes)
    if episodes % k:
        raise ValueError("episodes must be a multiple of envs_per_grid")
    per_env = episodes // k
    G = len(test_grids)
    env = BatchCoverageEnv(episode_config(env_config, True), G * k, grids=test_grids,
                           env_grid=np.repeat(np.arange(G, dtype=np.int32), k), device=device,
                           seed=seed, auto_reset=True, **env_kw)
    env.reset()
    out = generate_episodes(env, policy_factory(env), per_env)
    rewards = out["reward"].reshape(G, k * per_env)
    pcs = out["percent_covered"]
    env.close()
    return [float(r) for r in rewards.reshape(-1)], float(pcs.mean() * 100)


test_RLalg.__test__ = False  # not a pytest test (the reference's name)
