"""Diagnostic (round 6): the step-49 split/unsplit dist_obs mismatch of
test_c5_unsplit_transform_is_identical.  Runs both paths to step 49 (the
mass auto-reset at maxsteps 50), finds the maps whose dist_obs differ, and
checks each path's values there against the oracle (oracle/cpu_ref.py)
rebuilt from that path's own device state after step 48 and stepped with the
same actions.  Also dumps, per differing map, the device (M, witness), the
cache header and the full-list state, per path."""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import marlcov  # noqa: E402
from gpu_util import device_state, oracle_from_device  # noqa: E402
from marlcov import _lib  # noqa: E402
from test_gpu_parity import base_cfg  # noqa: E402

cfg = base_cfg(numrobot=16, dist_reward=1, maxsteps=50)
T = int(os.environ.get("DIAG_STEP", "49"))


def run(split):
    os.environ["MARLCOV_DIST_SPLIT"] = split
    env = marlcov.BatchCoverageEnv(cfg, 64, gen=dict(width=512, length=512, prob_obst=0.1, seed=1001), seed=9,
                                   auto_reset=True)
    env.reset()
    hist = []
    for t in range(T):
        env.step(env.random_actions(31, t))
        hist.append(env.dist_obs.clone())
    return env, hist


envs = {s: run(s) for s in ("1", "0")}
for t in range(T):
    if not torch.equal(envs["1"][1][t], envs["0"][1][t]):
        print(f"paths already differ at step {t}")
        break
else:
    print(f"paths identical through step {T - 1}")
pre = {}
for s, (env, _) in envs.items():
    pre[s] = {"mw": env.get_state(_lib.FIELD_DIST_MW).cpu().numpy().copy(),
              "pos": env.get_state(_lib.FIELD_POS).cpu().numpy().copy()}
acts = envs["1"][0].random_actions(31, T)
out = {}
for s, (env, _) in envs.items():
    env.step(acts)
    out[s] = env.dist_obs.cpu().numpy().copy()
    print(f"split={s}: listed {int(env.get_state(_lib.FIELD_DIST_LISTED).item())}, "
          f"totals {env.get_state(_lib.FIELD_DIST_TOTALS).cpu().tolist()}")
d = np.argwhere(out["1"] != out["0"])
print(f"step {T}: {len(d)} differing cells")
maps = sorted({(int(e), int(a)) for e, a, _, _ in d})
print("maps:", maps[:20], "..." if len(maps) > 20 else "")
# the oracle for the first few differing envs, rebuilt from each path's state before the step
a_h = acts.cpu().numpy()
for s, (env, _) in envs.items():
    pass
for (e, ag) in maps[:6]:
    cells = [(int(x), int(y)) for ee, aa, x, y in d if ee == e and aa == ag]
    print(f"env {e} agent {ag}: cells {cells[:6]}; split {[float(out['1'][e, ag, x, y]) for x, y in cells[:6]]} "
          f"unsplit {[float(out['0'][e, ag, x, y]) for x, y in cells[:6]]}")
    print(f"   pre-step (M, w): split {pre['1']['mw'][e, ag].tolist()} unsplit {pre['0']['mw'][e, ag].tolist()}")
# oracle check: rebuild from a fresh run to step T-1 (state equal in both paths through T-1)
os.environ["MARLCOV_DIST_SPLIT"] = "0"
env0 = marlcov.BatchCoverageEnv(cfg, 64, gen=dict(width=512, length=512, prob_obst=0.1, seed=1001), seed=9,
                                auto_reset=True)
env0.reset()
for t in range(T):
    env0.step(env0.random_actions(31, t))
sel = sorted({e for e, _ in maps[:6]})
st = device_state(env0, sel)
refs = {b: oracle_from_device(st, b, cfg) for b in sel}
env0.step(acts)
st1 = device_state(env0, sel)
for b in sel:
    o, r, dn = refs[b].step(a_h[b].astype(np.int64))
    if dn:
        p = st1["pos"][b]
        o, _ = refs[b].reset(False, None, positions=[tuple(q) for q in p])
    lay = np.asarray(o)[:, 3].astype(np.float32)
    for s in ("1", "0"):
        bad = np.argwhere(out[s][b] != lay)
        print(f"oracle env {b} (done={bool(dn)}): split={s} differs from the oracle at {len(bad)} cells",
              bad[:4].tolist())
