"""Load / replay the SuperGridRL golden fixtures (tests/golden/super/*.npz,
captured from the reference by tests/golden/make_golden_super.py) through any
class with the SuperGridRL interface: the CPU oracle or the HIP facade."""
from __future__ import annotations

import contextlib
import glob
import io
import json
import os

import numpy as np

SUPER_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "super")


def super_case_names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(SUPER_DIR, "*.npz")))


def load_super_case(name):
    z = np.load(os.path.join(SUPER_DIR, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


def super_grids(case):
    train = [g.astype(np.float64) for g in case["train"]]
    test = None
    if "num_test" in case:
        test = [case[f"test{i}"].astype(np.float64) for i in range(int(case["num_test"]))]
    return train, test


def make_super_env(env_cls, case, **kw):
    train, test = super_grids(case)
    np.random.seed(case["meta"]["seed"])
    with contextlib.redirect_stdout(io.StringIO()):
        return env_cls(train, dict(case["meta"]["config"]), test_set=test, **kw)


def super_action(case, t):
    kind = int(case["kind"][t])
    if kind == 0:
        return int(case["a_val"][t])
    if kind == 1:
        import torch
        return torch.tensor(int(case["a_val"][t]))
    if kind == 2:
        return None
    raise ValueError("reset event")


def replay_super(env, case, check):
    np.testing.assert_array_equal(env._xinds, case["init_x"])
    np.testing.assert_array_equal(env._yinds, case["init_y"])
    for t in range(len(case["kind"])):
        kind = int(case["kind"][t])
        with contextlib.redirect_stdout(io.StringIO()):
            if kind == 3:
                ind = int(case["r_ind"][t])
                (state, cur), _ = env.reset(bool(case["r_testing"][t]), None if ind < 0 else ind)
                reward = done = None
            else:
                (state, cur), reward, done = env.step(super_action(case, t))
        check(t, kind, state, cur, reward, done, case)


def check_super_golden(env):
    """Bit-exact comparison of every recorded field."""
    def check(t, kind, state, cur, reward, done, case):
        tag = f"{case['meta']['name']} event {t} kind {kind}"
        W, L = (int(v) for v in case["grid_shape"][t])
        state = np.asarray(state)
        assert state.dtype == np.float64 and state.shape == (int(case["state_layers"][t]), W, L), tag
        P = state.shape[0] - 3
        x, y = case["xinds"][t], case["yinds"][t]
        np.testing.assert_array_equal(env._xinds, x, err_msg=tag)
        np.testing.assert_array_equal(env._yinds, y, err_msg=tag)
        pos = np.zeros((P, W, L))
        if P == 1:
            pos[0][x, y] = 1
        else:
            pos[np.arange(P), x, y] = 1
        np.testing.assert_array_equal(state[:P], pos, err_msg=tag + " pos layers")
        free = np.unpackbits(case["free"][t], axis=-1)[:W, :L]
        obst = np.unpackbits(case["obst"][t], axis=-1)[:W, :L]
        np.testing.assert_array_equal(state[P], obst, err_msg=tag + " obstacles")
        np.testing.assert_array_equal(state[P + 1], free, err_msg=tag + " free")
        np.testing.assert_array_equal(state[P + 2], case["dist"][t][:W, :L].astype(np.float64),
                                      err_msg=tag + " distance layer")
        assert cur == case["currstep"][t], tag
        if kind != 3:
            assert float(reward) == case["reward"][t], (tag, float(reward), case["reward"][t])
            assert bool(done) == bool(case["done"][t]), tag
        assert env.percent_covered() == case["pc"][t], tag
        assert float(env._done_thresh) == case["done_thresh"][t], tag
        ap = -1 if env.a_prev is None else int(env.a_prev)
        assert ap == case["a_prev"][t], tag
    return check
