"""Capture the reference's known answer (SURVEY §8(c) pin 3).

The reference's only published result: the non-learning controllers BSA and
BA* cover 100 % of the hand-made test grids (``gridload(None)``,
``Utils/gridmaker.py:23-43``) in every test episode
(``Example_Experiments/Non_Learning/BA_Star/Example/TerminalOutput.txt:172-173``
says "100.0 percent"; the BSA log records the same runs).  The total reward
of each episode, 234 (205 free cells - 1 + 30 terminal), is NOT published:
it was captured by running the reference's own DecGridRL / BSA / BA* here,
in the build container, and is pinned by this fixture alone.

Runs ONLY in the build container, where the read-only reference checkout is
mounted at /root/reference.  It imports the reference's ``DecGridRL``,
``Policies.bsa.BSA``, ``Policies.ba_star.BA_Star`` and
``Utils.utils.generate_episode`` (with the same ``pygame`` / ``cv2`` stubs as
``make_golden.py``; neither is called on this path: no dist_reward, no
minimap, no render) and runs test episodes exactly as ``test_RLalg``
(``Utils/utils.py:111-149``) does, under the example configs
(``Example_Experiments/Non_Learning/{BSA,BA_Star}/Example/config.json``,
read here), one ``np.random.seed`` per episode.  It records, per episode: the
test grid index, the seed, the start cell, and per step the controller's
action, the reward, done and the next observation; plus the episode's
``percent_covered()`` and total reward.

The fixture (``tests/golden/known_answer.npz``) is inputs + outputs only.  The
replay tests (``tests/test_oracle_golden.py`` on the oracle,
``tests/test_gpu_parity.py`` on the HIP facade) feed the recorded actions and
require the recorded observation, reward and done at every step: equal
observations mean the controller, a deterministic function of them, would
have chosen the same actions.

    python tests/golden/make_known_answer.py
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, _install_stubs  # noqa: E402

POLICIES = ("bsa", "ba_star")
SEEDS = (0, 1, 2, 3)  # episodes per (policy, test grid)


def example_config(policy):
    d = {"bsa": "BSA", "ba_star": "BA_Star"}[policy]
    with open(os.path.join(REF, "Example_Experiments", "Non_Learning", d, "Example", "config.json")) as f:
        return json.load(f)


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    from Environments.dec_grid_rl import DecGridRL
    from Policies.ba_star import BA_Star
    from Policies.bsa import BSA
    from Utils.gridmaker import gridload
    from Utils.utils import generate_episode

    with contextlib.redirect_stdout(io.StringIO()):
        train_set, test_set = gridload(None)
    out = {}
    for pname in POLICIES:
        conf = example_config(pname)
        env_config, pc = conf["env_config"], conf["policy_config"]
        assert conf["grid_config"]["gridload"] == 1 and conf["grid_config"]["grid_dir"] == 0
        env = DecGridRL(train_set, env_config, use_graph=pc["use_graph"], test_set=test_set)
        if pname == "bsa":  # grid_rl_main.py:205-209
            policy = BSA(pc["internal_grid_rad"])
        else:
            policy = BA_Star(pc["internal_grid_rad"], env_config["egoradius"])
        ep_grid, ep_seed, ep_start, ep_len, ep_pc, ep_total = [], [], [], [], [], []
        acts, rews, dones, obs, obs0 = [], [], [], [], []
        for ind in range(len(test_set)):
            for seed in SEEDS:
                np.random.seed(seed)
                sink = io.StringIO()
                with contextlib.redirect_stdout(sink):
                    # the start cell is drawn by reset() inside generate_episode;
                    # replay the same draw to record it
                    st = np.random.get_state()
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
                print(f"{pname} grid {ind} seed {seed}: start {start}, {len(episode)} steps, "
                      f"total reward {total}, percent_covered {pcov}")
        out[f"{pname}__env_config"] = np.frombuffer(json.dumps(env_config, sort_keys=True).encode(), np.uint8)
        out[f"{pname}__ep_grid"] = np.array(ep_grid, np.int32)
        out[f"{pname}__ep_seed"] = np.array(ep_seed, np.int32)
        out[f"{pname}__ep_start"] = np.array(ep_start, np.int32)
        out[f"{pname}__ep_len"] = np.array(ep_len, np.int32)
        out[f"{pname}__ep_pc"] = np.array(ep_pc, np.float64)
        out[f"{pname}__ep_total"] = np.array(ep_total, np.float64)
        out[f"{pname}__obs0"] = np.stack(obs0)
        out[f"{pname}__actions"] = np.array(acts, np.int8)
        out[f"{pname}__rewards"] = np.array(rews, np.float64)
        out[f"{pname}__dones"] = np.array(dones, np.uint8)
        out[f"{pname}__obs"] = np.stack(obs)
    out["test_grids"] = np.stack(test_set).astype(np.int8)
    out["train_grids"] = np.stack(train_set).astype(np.int8)
    path = os.path.join(HERE, "known_answer.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
