"""Capture golden vectors from the real reference SuperGridRL.

Runs ONLY in the build container, where the read-only reference checkout is
mounted at /root/reference.  It imports ``Environments.super_grid_rl.SuperGridRL``
with the same two stubs as make_golden.py: ``pygame`` (ctor / render no-ops)
and ``cv2`` whose only member used on this path, ``distanceTransform``
(``super_grid_rl.py:294-296``, called by every ``get_state``), is the exact-L1
SciPy restatement — parity with real OpenCV stays unpinned.  Fixtures
(``tests/golden/super/*.npz``) hold inputs and outputs only.

    python tests/golden/make_golden_super.py
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "super")
sys.path.insert(0, HERE)

from make_golden import REF, _install_stubs, bernoulli, tri_valued  # noqa: E402

BASE = dict(numrobot=1, train_maxsteps=1000, test_maxsteps=1000, collision_penalty=5,
            senseradius=1, free_penalty=0.2, done_thresh=1, done_incr=0, terminal_reward=30,
            dist_reward=0, use_scanning=0)


def cfg(**kw):
    c = dict(BASE)
    c.update(kw)
    return c


def joint(rs, n, T):
    return [("int", int(sum(int(d) * 4 ** i for i, d in enumerate(rs.randint(0, 4, size=n)))))
            for _ in range(T)]


def build_cases():
    rs = np.random.RandomState(4321)
    cases = []

    def add(name, config, train, test=None, seed=0, events=()):
        cases.append(dict(name=name, config=config, train=train, test=test, seed=seed,
                          events=list(events)))

    add("sg_n1_r1", cfg(), [bernoulli(rs, 20, 20, 0.2)], seed=1, events=joint(rs, 1, 80))
    add("sg_n4_scan_dist_r2", cfg(numrobot=4, senseradius=2, free_penalty=0.3, dist_reward=1,
                                  use_scanning=1),
        [bernoulli(rs, 24, 30, 0.15)], seed=2, events=joint(rs, 4, 90))
    add("sg_n3_dist_noscan_done_incr", cfg(numrobot=3, free_penalty=0.1, dist_reward=1,
                                           done_thresh=0.3, done_incr=0.2),
        [bernoulli(rs, 14, 14, 0.1)], seed=3, events=joint(rs, 3, 120))
    add("sg_zero_cells_n2_r2", cfg(numrobot=2, senseradius=2, free_penalty=0.7, dist_reward=1),
        [tri_valued(rs, 22, 18)], seed=4, events=joint(rs, 2, 70))
    ev = []
    specials = [("int", -1), ("none",), ("int", 4 ** 2 + 5), ("tensor", 7), ("int", 2 * 4 ** 2 + 1),
                ("int", 3 * 4 ** 2 + 9), ("tensor", 4 ** 2 * 1 + 3)]
    for t in range(70):
        ev.append(specials[(t // 5) % len(specials)] if t % 5 == 4 else joint(rs, 2, 1)[0])
    add("sg_sentinels_quotients_n2", cfg(numrobot=2, dist_reward=1, collision_penalty=1.5),
        [bernoulli(rs, 16, 16, 0.2)], seed=5, events=ev)
    gs = [bernoulli(rs, 15, 15, 0.1) for _ in range(3)]
    ev = []
    for _ in range(3):
        ev.append(("reset", False, None))
        ev += joint(rs, 2, 25)
    add("sg_multi_episode_random_grid", cfg(numrobot=2, dist_reward=1, use_scanning=1), gs, seed=6,
        events=ev)
    add("sg_crowded_scan_n8", cfg(numrobot=8, use_scanning=1, collision_penalty=2, free_penalty=0.05),
        [bernoulli(rs, 9, 9, 0.25)], seed=7, events=joint(rs, 8, 50))
    add("sg_n16_joint", cfg(numrobot=16, senseradius=2, dist_reward=1),
        [bernoulli(rs, 40, 40, 0.1)], seed=8, events=joint(rs, 16, 20))
    ev = []
    for ind in range(2):
        ev.append(("reset", True, ind))
        ev += joint(rs, 1, 40)
    add("sg_test_set_r3", cfg(senseradius=3, dist_reward=1, free_penalty=0.25),
        [bernoulli(rs, 18, 26, 0.1)], test=[bernoulli(rs, 18, 26, 0.2), bernoulli(rs, 12, 12, 0.0)],
        seed=9, events=ev)
    return cases


def run_case(SuperGridRL, case):
    import torch

    np.random.seed(case["seed"])
    env = SuperGridRL(case["train"], case["config"], test_set=case["test"])
    rec = {k: [] for k in ("kind", "a_val", "r_testing", "r_ind", "reward", "done", "xinds", "yinds",
                           "free", "obst", "dist", "pc", "currstep", "done_thresh", "a_prev", "grid_shape",
                           "state_layers")}
    init = dict(x=env._xinds.copy(), y=env._yinds.copy())
    for ev in case["events"]:
        kind = ev[0]
        a_val, r_t, r_i = 0, 0, -1
        if kind == "reset":
            state, _grid = env.reset(ev[1], ev[2])
            reward, done, code = np.nan, False, 3
            r_t, r_i = int(bool(ev[1])), (-1 if ev[2] is None else int(ev[2]))
        else:
            if kind == "int":
                action, code, a_val = ev[1], 0, ev[1]
            elif kind == "tensor":
                action, code, a_val = torch.tensor(ev[1]), 1, ev[1]
            else:
                action, code = None, 2
            state, reward, done = env.step(action)
            assert isinstance(done, (bool, np.bool_)), type(done)
        arr, cur = state
        assert cur == env._currstep
        P = arr.shape[0] - 3
        pos = np.zeros_like(arr[:P])
        if env._use_scanning:
            pos[0][env._xinds, env._yinds] = 1
        else:
            pos[np.arange(P), env._xinds, env._yinds] = 1
        np.testing.assert_array_equal(arr[:P], pos)  # layers 0..P-1 follow from (x, y)
        np.testing.assert_array_equal(arr[P], env._observed_obstacles)
        np.testing.assert_array_equal(arr[P + 1], env._free)
        rec["kind"].append(code)
        rec["a_val"].append(a_val)
        rec["r_testing"].append(r_t)
        rec["r_ind"].append(r_i)
        rec["reward"].append(float(reward))
        rec["done"].append(bool(done))
        rec["xinds"].append(env._xinds.copy())
        rec["yinds"].append(env._yinds.copy())
        W, L = env._gridwidth, env._gridlen
        pad = lambda a: np.pad(a, ((0, 64 - W), (0, 64 - L)))  # noqa: E731  fixed shape for stacking
        assert W <= 64 and L <= 64
        rec["free"].append(np.packbits(pad(env._free).astype(np.uint8), axis=-1))
        rec["obst"].append(np.packbits(pad(env._observed_obstacles).astype(np.uint8), axis=-1))
        d = arr[P + 2]
        assert np.all(d.astype(np.float32).astype(np.float64) == d)
        rec["dist"].append(pad(d).astype(np.float32))
        rec["pc"].append(env.percent_covered())
        rec["currstep"].append(env._currstep)
        rec["done_thresh"].append(float(env._done_thresh))
        rec["a_prev"].append(-1 if env.a_prev is None else int(env.a_prev))
        rec["grid_shape"].append((W, L))
        rec["state_layers"].append(arr.shape[0])
    return rec, init


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    from Environments.super_grid_rl import SuperGridRL  # noqa: E402

    os.makedirs(OUT, exist_ok=True)
    total = 0
    for case in build_cases():
        with contextlib.redirect_stdout(io.StringIO()):  # done() prints
            rec, init = run_case(SuperGridRL, case)
        meta = dict(name=case["name"], config=case["config"], seed=case["seed"])
        arrays = dict(meta=np.array(json.dumps(meta)),
                      train=np.stack([g.astype(np.int8) for g in case["train"]]),
                      init_x=init["x"], init_y=init["y"])
        if case["test"] is not None:
            shapes = {g.shape for g in case["test"]}
            for i, g in enumerate(case["test"]):
                arrays[f"test{i}"] = g.astype(np.int8)
            arrays["num_test"] = np.array(len(case["test"]))
            del shapes
        for k, v in rec.items():
            arrays[k] = np.stack([np.asarray(x) for x in v])
        path = os.path.join(OUT, case["name"] + ".npz")
        np.savez_compressed(path, **arrays)
        total += os.path.getsize(path)
        print(f"{case['name']:36s} events={len(case['events']):4d} {os.path.getsize(path)/1024:7.1f} KiB")
    print(f"total {total/1024:.1f} KiB")


if __name__ == "__main__":
    main()
