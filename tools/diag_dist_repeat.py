"""Diagnostic: C5 dist_obs / max(d) of the split and the unsplit transform
paths (MARLCOV_DIST_SPLIT) over repeated identical runs; prints the first
step where two runs differ."""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import marlcov  # noqa: E402
from marlcov import _lib  # noqa: E402
from test_gpu_parity import base_cfg  # noqa: E402

cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=50)


def run(split):
    os.environ["MARLCOV_DIST_SPLIT"] = split
    env = marlcov.BatchCoverageEnv(cfg, 64, gen=dict(width=512, length=512, prob_obst=0.1, seed=1001), seed=9,
                                   auto_reset=True)
    env.reset()
    acc = []
    for t in range(60):
        env.step(env.random_actions(31, t))
        mw = env.get_state(_lib.FIELD_DIST_MW).clone()
        acc.append((env.dist_obs.clone(), mw, env.get_state(_lib.FIELD_DIST_LISTED).item()))
    del env
    return acc


runs = [("1", run("1")), ("0", run("0")), ("1", run("1")), ("0", run("0"))]
base = runs[0][1]
for name, acc in runs[1:]:
    for t in range(60):
        a, b = base[t], acc[t]
        if not torch.equal(a[0], b[0]):
            d = (a[0] != b[0]).nonzero()
            e, ag = int(d[0, 0]), int(d[0, 1])
            print(f"split={name} step {t}: dist_obs differs at {d.shape[0]} cells, first env {e} agent {ag}; "
                  f"(M, w) {a[1][e, ag].tolist()} vs {b[1][e, ag].tolist()}; listed {a[2]} vs {b[2]}")
            print("   cells:", d[:4].tolist(), a[0][tuple(d[0].tolist())].item(), b[0][tuple(d[0].tolist())].item())
            break
    else:
        print(f"split={name}: identical dist_obs over 60 steps")

# the true max(d) of every map at step 49 of each path, from the device's own
# free planes (oracle restatement of the transform)
import numpy as np  # noqa: E402
from gpu_util import device_state  # noqa: E402
from oracle.cpu_ref import l1_distance_to_covered  # noqa: E402


def check(split, steps=50, envs=(2, 26, 27, 34)):
    os.environ["MARLCOV_DIST_SPLIT"] = split
    env = marlcov.BatchCoverageEnv(cfg, 64, gen=dict(width=512, length=512, prob_obst=0.1, seed=1001), seed=9,
                                   auto_reset=True)
    env.reset()
    for t in range(steps):
        env.step(env.random_actions(31, t))
    mw = env.get_state(_lib.FIELD_DIST_MW).cpu().numpy()
    st = device_state(env, list(envs))
    bad = 0
    for b in envs:
        for i in range(16):
            M = int(mw[b, i, 0])
            if M < 0:
                continue
            fp = np.pad(st["free"][b][i], 2)
            true = int(l1_distance_to_covered(fp).max())
            if true != M:
                bad += 1
                print(f"  split={split} env {b} agent {i}: device M {M}, true {true}")
    print(f"split={split}: {bad} wrong M among envs {envs}")


check("1")
check("0")
