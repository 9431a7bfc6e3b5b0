"""Helpers to load the golden fixtures and replay them through any env class
with the DecGridRL interface (the CPU oracle or the HIP-backed facade)."""
from __future__ import annotations

import contextlib
import glob
import io
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))
                  if not os.path.basename(p).startswith(("beam_tables", "known_answer", "bg2_")))


def load_case(name):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


def grids(case, key):
    if key not in case:
        return None
    return [g.astype(np.float64) for g in case[key]]


def event_action(case, t):
    kind = int(case["kind"][t])
    if kind == 0:
        return int(case["meta"]["a_int_digits"][t])
    if kind == 1:
        n = case["xinds"].shape[1]
        return np.array(case["a_vec"][t][:max(1, n)])
    if kind == 2:
        return None
    raise ValueError("reset event")


def unpack(packed, width):
    return np.unpackbits(packed, axis=-1)[..., :width]


def make_env(env_cls, case, **kw):
    meta = case["meta"]
    np.random.seed(meta["seed"])
    config = dict(meta["config"])
    if meta["even_beams"] is not None:
        config["allow_even_beams"] = True
    with contextlib.redirect_stdout(io.StringIO()):
        env = env_cls(grids(case, "train"), config, use_graph=meta["use_graph"],
                      test_set=grids(case, "test"), **kw)
    if meta["even_beams"] is not None:
        th = np.linspace(0, 2 * np.pi, meta["even_beams"], endpoint=False)
        env._sensor.set_thetalist(th)
    return env


def replay(env, case, check, max_events=None):
    """Replay a golden case; ``check(t, kind, out, case)`` compares step t."""
    meta = case["meta"]
    comm = bool(meta["config"]["allow_comm"] and meta["use_graph"])
    n_ev = len(case["kind"]) if max_events is None else min(max_events, len(case["kind"]))
    for t in range(n_ev):
        kind = int(case["kind"][t])
        with contextlib.redirect_stdout(io.StringIO()):
            if kind == 3:
                testing = bool(case["r_testing"][t])
                ind = int(case["r_ind"][t])
                out = env.reset(testing, None if ind < 0 else ind)
                obs, reward, done = out[0], None, None
            else:
                out = env.step(event_action(case, t))
                obs = out[0][0] if comm else out[0]
                reward, done = out[1], out[2]
        check(t, kind, dict(obs=obs, reward=reward, done=done, raw=out), case)


def check_against_golden(env):
    """Bit-exact comparison of env (oracle or facade) with the golden record."""
    def check(t, kind, out, case):
        tag = f"{case['meta']['name']} event {t} kind {kind}"
        np.testing.assert_array_equal(np.asarray(out["obs"], dtype=np.float64), case["obs"][t],
                                      err_msg=tag + " obs")
        if kind != 3:
            r = float(out["reward"])
            assert r == case["reward"][t], (tag, r, case["reward"][t])
            assert bool(out["done"]) == bool(case["done"][t]), tag
        np.testing.assert_array_equal(env._xinds, case["xinds"][t], err_msg=tag)
        np.testing.assert_array_equal(env._yinds, case["yinds"][t], err_msg=tag)
        snap = env.snapshot()
        for key, gkey in (("free_pad", "free"), ("obst_pad", "obst"), ("robot_pad", "robot"),
                          ("visited", "visited")):
            np.testing.assert_array_equal(np.packbits(snap[key], axis=-1), case[gkey][t],
                                          err_msg=f"{tag} {key}")
        np.testing.assert_array_equal(snap["adjacency"], case["adj"][t], err_msg=tag + " adj")
        assert env.percent_covered() == case["pc"][t], tag
        assert snap["currstep"] == case["currstep"][t], tag
        assert snap["done_thresh"] == case["done_thresh"][t], tag
        np.testing.assert_array_equal(env._grid.astype(np.int8), case["grid"][t], err_msg=tag)
    return check





# ---------------------------------------------------------------------------
# The reference's published known answer (SURVEY 8(c) pin 3): BSA / BA* test
# episodes on the hand-made grids, captured by tests/golden/make_known_answer.py
# ---------------------------------------------------------------------------
KNOWN_ANSWER_POLICIES = ("bsa", "ba_star")


def load_known_answer(name="known_answer.npz"):
    z = np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False)
    return {k: z[k] for k in z.files}


def replay_known_answer(env_cls, ka, policy, expect=(234.0, 1.0)):
    """Replay every recorded test episode of ``policy`` through ``env_cls``
    (the oracle or the HIP facade) the way ``test_RLalg`` runs it
    (Utils/utils.py:6-44,111-149): one env over the hand-made test grids,
    ``np.random.seed(seed)`` then ``reset(True, ind)``, then the controller's
    recorded actions.  Observation, reward and done must equal the record at
    every step; each episode must end done with the recorded total reward and
    percent_covered(), which must be ``expect`` when given (BSA / BA*: 234
    and 1.0).  A record with ``<policy>__max_steps`` was cut there (the
    capture lowered ``_test_maxsteps``, generate_episode's cut).  Returns the
    per-episode (total reward, percent covered)."""
    pre = policy + "__"
    config = json.loads(ka[pre + "env_config"].tobytes().decode())
    test = [g.astype(np.float64) for g in ka["test_grids"]]
    train = [g.astype(np.float64) for g in ka["train_grids"]]
    with contextlib.redirect_stdout(io.StringIO()):
        env = env_cls(train, config, use_graph=False, test_set=test)
    if pre + "max_steps" in ka:
        env._test_maxsteps = int(ka[pre + "max_steps"])
    n_ep = len(ka[pre + "ep_len"])
    off = np.concatenate([[0], np.cumsum(ka[pre + "ep_len"])])
    results = []
    for e in range(n_ep):
        ind, seed = int(ka[pre + "ep_grid"][e]), int(ka[pre + "ep_seed"][e])
        tag = f"{policy} episode {e} (test grid {ind}, seed {seed})"
        np.random.seed(seed)
        with contextlib.redirect_stdout(io.StringIO()):
            obs, grid = env.reset(True, ind)
        np.testing.assert_array_equal(grid, np.pad(test[ind], 1, constant_values=-1), err_msg=tag)
        assert (int(env._xinds[0]), int(env._yinds[0])) == tuple(ka[pre + "ep_start"][e]), tag
        np.testing.assert_array_equal(np.asarray(obs[0], np.float64), ka[pre + "obs0"][e], err_msg=tag + " reset obs")
        total, done, steps = 0.0, False, 0
        for t in range(off[e], off[e + 1]):
            assert not done, (tag, "record continues after done")
            with contextlib.redirect_stdout(io.StringIO()):
                obs, r, done = env.step(int(ka[pre + "actions"][t]))
            steps += 1
            stag = f"{tag} step {steps}"
            np.testing.assert_array_equal(np.asarray(obs[0], np.float64), ka[pre + "obs"][t], err_msg=stag + " obs")
            assert float(r) == float(ka[pre + "rewards"][t]), (stag, float(r), float(ka[pre + "rewards"][t]))
            assert bool(done) == bool(ka[pre + "dones"][t]), stag
            if env._currstep == env._test_maxsteps:  # utils.py:20-21
                done = True
            total += r
        pc = env.percent_covered()
        assert done, tag
        assert total == ka[pre + "ep_total"][e], (tag, total)
        assert pc == ka[pre + "ep_pc"][e], (tag, pc)
        if expect is not None:
            assert (total, pc) == expect, (tag, total, pc)
        results.append((total, pc))
    return results
