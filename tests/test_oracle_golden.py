"""Pin the CPU oracle (oracle/cpu_ref.py) against golden vectors captured from
the real reference (tests/golden/make_golden.py).  Bit-exact on every field."""
import numpy as np
import pytest

from golden_util import case_names, load_case, make_env, replay, GOLDEN_DIR
from oracle.cpu_ref import DecGridRLRef, lidar_beam_table, lidar_thetas


def check_against_golden(env):
    def check(t, kind, out, case):
        tag = f"{case['meta']['name']} event {t} kind {kind}"
        np.testing.assert_array_equal(np.asarray(out["obs"], dtype=np.float64), case["obs"][t], err_msg=tag)
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
        np.testing.assert_array_equal(snap["adjacency"], case["adj"][t], err_msg=tag)
        assert env.percent_covered() == case["pc"][t], tag
        assert snap["currstep"] == case["currstep"][t], tag
        assert snap["done_thresh"] == case["done_thresh"][t], tag
        np.testing.assert_array_equal(env._grid.astype(np.int8), case["grid"][t], err_msg=tag)
    return check


@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference_golden(name):
    case = load_case(name)
    env = make_env(DecGridRLRef, case)
    replay(env, case, check_against_golden(env))


def test_beam_table_bits():
    z = np.load(GOLDEN_DIR + "/beam_tables.npz")
    for key in z.files:
        b = int(key[1:])
        tab = lidar_beam_table(lidar_thetas(b))
        np.testing.assert_array_equal(tab.view(np.uint64), z[key].view(np.uint64), err_msg=key)


def test_golden_inventory():
    names = case_names()
    assert len(names) >= 20
    for must in ("c1_empty32", "lidar_n4_48", "lidar_360_r20", "joint_n16",
                 "sentinels_and_odd_actions", "map_sharing_n4", "comm_graph_n4"):
        assert must in names
