"""Calibrate the CPU baseline: time the REFERENCE's DecGridRL.step against the
oracle restatement (oracle/cpu_ref.py) on one core, same configs and actions.

    python tools/calibrate_cpu.py [--secs 8] [--configs c1,c2,c4,c5] [--out profiles/r3/cpu_calibration.json]

Runs ONLY in the build container: it imports the read-only reference checkout
(/root/reference, or $MARLCOV_REFERENCE) with the pygame / cv2 stubs of
tests/golden/make_golden.py; the reference never travels to
the GPU box.  bench.py's cpu_baseline times the oracle ("kind": "port") on the
GPU box's cores; the ratio printed here says how the port's rate relates to
the reference's own step on the same core (> 1: the port is faster).

Each config is timed in one process pinned to one core, the reference and the
port alternating in rounds of ``--secs`` each (3 rounds), so clock drift hits
both; the median rate of each side is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

BASE = dict(maxsteps=1000, collision_penalty=5, done_thresh=1, done_incr=0, terminal_reward=30, dist_reward=0,
            train_maxsteps=1000, test_maxsteps=1000, egoradius=2, mini_map_rad=0, comm_radius=0, allow_comm=0,
            map_sharing=0, single_square_tool=0, dijkstra_input=0, sensor_type="lidar")
# SURVEY §8(d) configs (C1: empty 32x32, one agent; the others Bernoulli 0.1)
CONFIGS = {
    "c1": dict(numrobot=1, width=32, p=0.0, sensor_config={"num_lasers": 21, "range": 10}),
    "c2": dict(numrobot=4, width=128, p=0.1, sensor_config={"num_lasers": 21, "range": 10}),
    "c4": dict(numrobot=8, width=256, p=0.1, sensor_config={"num_lasers": 360, "range": 20}, even=True),
    "c5": dict(numrobot=16, width=512, p=0.1, sensor_config={"num_lasers": 21, "range": 10},
               extra={"dist_reward": 1}, maxsteps=2000),
}


def make_cfg(c):
    cfg = dict(BASE, numrobot=c["numrobot"], sensor_config=dict(c["sensor_config"]), **c.get("extra", {}))
    if "maxsteps" in c:
        cfg["maxsteps"] = c["maxsteps"]
    return cfg


def build_reference_env(cls, grid, cfg, even):
    import numpy as np
    if even:  # lidar.py:11 asserts an odd count: build with B+1, then set B
        n = cfg["sensor_config"]["num_lasers"]
        c2 = dict(cfg, sensor_config=dict(cfg["sensor_config"], num_lasers=n + 1))
        env = cls([grid], c2)
        env._sensor._num_lasers = n
        env._sensor._thetalist = np.linspace(0, 2 * np.pi, n, endpoint=False)
        return env
    return cls([grid], cfg)


def timed(env, acts, secs):
    n, t0 = 0, time.perf_counter()
    while True:
        _, _, done = env.step(acts[n % len(acts)])
        n += 1
        if done:
            env.reset(False, None)
        if n % 4 == 0 and time.perf_counter() - t0 >= secs:
            return n / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=8.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--configs", default="c1,c2,c4,c5")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r3", "cpu_calibration.json"))
    args = ap.parse_args()
    try:
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[0]})
    except (AttributeError, OSError):
        pass
    import numpy as np
    from make_golden import _load_reference

    RefDecGridRL, _ = _load_reference()
    from oracle.cpu_ref import DecGridRLRef

    results = {}
    for name in args.configs.split(","):
        c = CONFIGS[name]
        cfg = make_cfg(c)
        rs = np.random.RandomState(1000)
        W = c["width"]
        grid = rs.choice([1.0, -1.0], size=(W, W), p=[1 - c["p"], c["p"]]) if c["p"] > 0 else np.ones((W, W))
        # joint actions as Python ints (base 4, robot 0 = LSD, dec_grid_rl.py:110-115): the
        # reference raises on per-agent ndarrays for N > 1
        digits = rs.randint(0, 4, size=(4096, c["numrobot"]))
        acts = [int(sum(int(d) * 4 ** i for i, d in enumerate(row))) for row in digits]
        np.random.seed(0)
        ref = build_reference_env(RefDecGridRL, grid, cfg, c.get("even", False))
        np.random.seed(0)
        port = DecGridRLRef([grid], dict(cfg, allow_even_beams=c.get("even", False)))
        rr, pr = [], []
        for _ in range(args.rounds):
            rr.append(timed(ref, acts, args.secs))
            pr.append(timed(port, acts, args.secs))
        r, p = float(np.median(rr)), float(np.median(pr))
        results[name] = {"reference_env_steps_per_s": round(r, 2), "port_env_steps_per_s": round(p, 2),
                         "port_over_reference": round(p / r, 3), "rounds": args.rounds, "secs_per_round": args.secs,
                         "reference_rounds": [round(x, 2) for x in rr], "port_rounds": [round(x, 2) for x in pr]}
        print(f"{name}: reference {r:10.2f}  port {p:10.2f}  port/reference {p / r:.3f}", flush=True)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except (OSError, StopIteration):
        pass
    out = {"what": "reference DecGridRL.step (imported, pygame/cv2 stubs; cv2.distanceTransform restated with "
                   "scipy taxicab for C5) vs oracle/cpu_ref.py DecGridRLRef.step, one env, one pinned core, "
                   "same grid / actions / seeds, alternating rounds",
           "host_cpu": cpu, "numpy": np.__version__, "results": results}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
