"""Capture a golden from the reference on its own shipped maps (Grids/bg2_*).

Runs ONLY in the build container, where the read-only reference checkout is
mounted at /root/reference.  Imports the reference's ``DecGridRL``,
``Policies.stc.STC``, ``Utils.gridmaker.gridload`` and
``Utils.utils.generate_episode`` with the same ``pygame`` / ``cv2`` stubs as
``make_golden.py`` (neither is called on this path: no dist_reward, no
minimap, no render).

1. The map fixtures (``tests/golden/maps/``): the two first files by name of
   ``Grids/bg2_100x100`` and the first of ``Grids/bg2_1073x1073``, copied as
   data (mode ``L`` PNGs, values {0, 255}).
2. ``bg2_100x100_stc.npz``: the STC example
   (``Example_Experiments/Non_Learning/STC/Example/config.json``: 1 robot,
   square sensor r=2, single_square_tool, STC with internal_grid_rad 105) on
   those two maps, loaded by the reference's own ``gridload``
   (``gridmaker.py:82-102``; two files give train = test = both,
   ``:96-98``).  Test episodes as ``test_RLalg`` runs them
   (``Utils/utils.py:111-149``), one ``np.random.seed`` per episode, cut at
   ``MAX_STEPS`` steps (the config's test_maxsteps is 100,000): per step the
   controller's action, reward, done and observation.  The grids the
   reference loaded are stored with it (so the replay does not depend on the
   filesystem's ``os.listdir`` order).

    python tests/golden/make_bg2_golden.py
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _install_stubs  # noqa: E402

MAPS = os.path.join(HERE, "maps")
MAX_STEPS = 1500
SEEDS = (0, 1)


def copy_maps():
    os.makedirs(MAPS, exist_ok=True)
    out = []
    for sub, n in (("bg2_100x100", 2), ("bg2_1073x1073", 1)):
        for name in sorted(os.listdir(os.path.join(REF, "Grids", sub)))[:n]:
            dst = os.path.join(MAPS, f"{sub}__{name}")
            shutil.copyfile(os.path.join(REF, "Grids", sub, name), dst)
            out.append(dst)
    return out



def main():
    copy_maps()
    _install_stubs()
    sys.path.insert(0, REF)
    from Environments.dec_grid_rl import DecGridRL
    from Policies.stc import STC
    from Utils.gridmaker import gridload
    from Utils.utils import generate_episode

    with open(os.path.join(REF, "Example_Experiments", "Non_Learning", "STC", "Example", "config.json")) as f:
        conf = json.load(f)
    env_config, pc = conf["env_config"], conf["policy_config"]
    with tempfile.TemporaryDirectory() as tmp:
        for p in sorted(os.listdir(MAPS)):
            if p.startswith("bg2_100x100__"):
                shutil.copyfile(os.path.join(MAPS, p), os.path.join(tmp, p.split("__", 1)[1]))
        gc = dict(conf["grid_config"], grid_dir=tmp)
        with contextlib.redirect_stdout(io.StringIO()):
            train_set, test_set = gridload(gc)
    assert len(train_set) == len(test_set) == 2
    np.random.seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        env = DecGridRL(train_set, env_config, use_graph=pc["use_graph"], test_set=test_set)
    env._test_maxsteps = MAX_STEPS
    policy = STC(pc["internal_grid_rad"])
    out = {}
    ep_grid, ep_seed, ep_start, ep_len, ep_pc, ep_total = [], [], [], [], [], []
    acts, rews, dones, obs, obs0 = [], [], [], [], []
    for ind in range(len(test_set)):
        for seed in SEEDS:
            np.random.seed(seed)
            st = np.random.get_state()
            with contextlib.redirect_stdout(io.StringIO()):
                episode, total = generate_episode(env, policy, None, testing=True, ind=ind)
                pcov = env.percent_covered()
            np.random.set_state(st)
            with contextlib.redirect_stdout(io.StringIO()):
                o0, _ = env.reset(True, ind)
            start = (int(env._xinds[0]), int(env._yinds[0]))
            ep_grid.append(ind)
            ep_seed.append(seed)
            ep_start.append(start)
            ep_len.append(len(episode))
            ep_pc.append(float(pcov))
            ep_total.append(float(total))
            obs0.append(np.asarray(o0[0], dtype=np.int8))
            for (s, a, r, ns, d) in episode:
                acts.append(int(a))
                rews.append(float(r))
                dones.append(bool(d))
                obs.append(np.asarray(ns, dtype=np.int8))
                assert np.array_equal(np.asarray(ns, dtype=np.int8), ns)
            print(f"stc grid {ind} seed {seed}: start {start}, {len(episode)} steps, total reward {total}, "
                  f"percent_covered {pcov}")
    p = "stc"
    out[f"{p}__env_config"] = np.frombuffer(json.dumps(env_config, sort_keys=True).encode(), np.uint8)
    out[f"{p}__max_steps"] = np.array(MAX_STEPS, np.int32)
    out[f"{p}__ep_grid"] = np.array(ep_grid, np.int32)
    out[f"{p}__ep_seed"] = np.array(ep_seed, np.int32)
    out[f"{p}__ep_start"] = np.array(ep_start, np.int32)
    out[f"{p}__ep_len"] = np.array(ep_len, np.int32)
    out[f"{p}__ep_pc"] = np.array(ep_pc, np.float64)
    out[f"{p}__ep_total"] = np.array(ep_total, np.float64)
    out[f"{p}__obs0"] = np.stack(obs0)
    out[f"{p}__actions"] = np.array(acts, np.int8)
    out[f"{p}__rewards"] = np.array(rews, np.float64)
    out[f"{p}__dones"] = np.array(dones, np.uint8)
    out[f"{p}__obs"] = np.stack(obs)
    out["test_grids"] = np.stack(test_set).astype(np.int8)
    out["train_grids"] = np.stack(train_set).astype(np.int8)
    path = os.path.join(HERE, "bg2_100x100_stc.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
