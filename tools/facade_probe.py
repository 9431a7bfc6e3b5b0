"""Single-env facade step rate (marlcov.DecGridRL, the reference's own
interface, one env per handle) next to the oracle restatement's step on the
same episode: what a BSA / BA*-style controller calling env.step() in a loop
sees.  C2-shaped env (4 agents, 128x128, lidar 21 beams R=10).

    python tools/facade_probe.py [--steps 300]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    import marlcov
    from oracle.cpu_ref import DecGridRLRef
    cfg = dict(numrobot=4, maxsteps=100000, collision_penalty=5, done_thresh=1, done_incr=0,
               terminal_reward=30, dist_reward=0, train_maxsteps=100000, test_maxsteps=100000,
               egoradius=2, mini_map_rad=0, comm_radius=0, allow_comm=0, map_sharing=0,
               single_square_tool=0, dijkstra_input=0, sensor_type="lidar",
               sensor_config={"num_lasers": 21, "range": 10})
    rs = np.random.RandomState(3)
    grid = np.where(rs.rand(128, 128) < 0.1, -1.0, 1.0)
    acts = np.random.RandomState(4).randint(0, 4 ** 4, size=args.steps)
    out = {}
    for name, cls in (("facade", marlcov.DecGridRL), ("oracle", DecGridRLRef)):
        np.random.seed(11)
        env = cls([grid], cfg)
        env.reset(False, 0)
        for a in acts[:10]:
            env.step(int(a))
        t0 = time.perf_counter()
        for a in acts:
            env.step(int(a))
        dt = time.perf_counter() - t0
        out[name] = {"steps_per_s": round(args.steps / dt, 1), "us_per_step": round(dt / args.steps * 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
