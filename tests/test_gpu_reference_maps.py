"""The reference's own shipped maps on the device (Grids/bg2_*, copies in
tests/golden/maps; SURVEY 8(f) rank 4, gridmaker.py:82-102).

* The STC example (Example_Experiments/Non_Learning/STC/Example/config.json)
  on two bg2_100x100 maps: the controller's test episodes captured from the
  reference (tests/golden/make_bg2_golden.py) replay through the HIP facade
  with observation, reward and done equal every step.
* A bg2_1073x1073 map (the grid-size scaling axis) stepped in a
  batch against the oracle, at the C2 and C4 sensor configs.
* dist_reward on that map (1,079 extended rows: the big-map distance
  kernel, mc_dist.hip dist_big_kernel) against the oracle, (M, witness) of
  every map checked against a fresh transform; a grid past the big kernel's
  1,088 rows is rejected by mc_create with a message.
"""
import os

import numpy as np
import pytest

from golden_util import GOLDEN_DIR, load_known_answer, replay_known_answer
from test_gpu_parity import base_cfg
from test_gpu_shapes import run_against_oracle

pytestmark = pytest.mark.gpu

MAPS = os.path.join(GOLDEN_DIR, "maps")


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


def big_map():
    """bg2_1073x1073/AR0011SR.png as the reference's gridload makes it:
    float64, 0 -> -1, 255 -> 1 (gridmaker.py:89-91)."""
    import marlcov
    _, test = marlcov.gridload({"grid_dir": MAPS, "numgrids": 1000}, sort=True)
    grids = [g for g in test if g.shape == (1073, 1073)]
    assert len(grids) == 1
    return grids[0]


def test_facade_bg2_stc_replay(torch_cuda):
    """STC on bg2_100x100 (square sensor r=2, single_square_tool, 1 robot):
    4 recorded test episodes (2 maps x 2 seeds, 288-1,276 steps, some ending
    on the controller's -1 sentinel) replay through the HIP facade bit for
    bit, ending with the recorded total reward and percent_covered()."""
    import marlcov
    ka = load_known_answer("bg2_100x100_stc.npz")
    res = replay_known_answer(marlcov.DecGridRL, ka, "stc", expect=None)
    assert len(res) == 4


@pytest.mark.parametrize("shape", ["c2", "c4"])
def test_bg2_1073_batch_matches_oracle(torch_cuda, shape):
    """Four envs on one 1073x1073 reference map (1,075 padded rows), every env
    tracked by the oracle from the reset through 30 steps with auto-resets
    (maxsteps 12): obs, reward, done, positions, maps and counters."""
    import marlcov
    torch = torch_cuda
    if shape == "c2":
        cfg = base_cfg(numrobot=4, maxsteps=12)
    else:
        cfg = base_cfg(numrobot=8, maxsteps=12, allow_even_beams=True,
                       sensor_config={"num_lasers": 360, "range": 20})
    g = big_map()
    B = 4
    env = marlcov.BatchCoverageEnv(cfg, B, grids=[g], auto_reset=True, seed=3, env_offset=0)
    env.reset()
    resets = run_against_oracle(torch, env, cfg, np.random.RandomState(1073), 30, list(range(B)), 3,
                                f"bg2_1073 {shape}", sentinel_p=0.02)
    assert resets >= B


def test_bg2_1073_dist_reward_matches_oracle(torch_cuda):
    """dist_reward (the C5 frontier reward) on the 1073x1073 reference map:
    1,079 extended rows, past the LDS-bitboard transform's 832, so every
    listed map runs the big-map kernel (no top-cell cache).  Two envs x 4
    agents tracked by the oracle from the reset through 16 steps with an
    auto-reset (maxsteps 8): reward with the float32 distance terms, the
    float distance obs layer, maps, and every known (M, witness) against a
    fresh transform (dec_grid_rl.py:222-223,239-240,260-282)."""
    import marlcov
    from marlcov import _lib
    torch = torch_cuda
    assert _lib.load().mc_build_param(_lib.PARAM_DIST_MAX_ROWS) == 1088
    cfg = base_cfg(numrobot=4, dist_reward=1, maxsteps=8)
    env = marlcov.BatchCoverageEnv(cfg, 2, grids=[big_map()], auto_reset=True, seed=5)
    env.reset()
    resets = run_against_oracle(torch, env, cfg, np.random.RandomState(79), 16, [0, 1], 5, "bg2_1073 dist",
                                dist_check=True, sentinel_p=0.0)
    assert resets >= 2


def test_dist_reward_rows_past_the_big_kernel_are_rejected(torch_cuda):
    """Extended grids past the big-map kernel's 1,088 rows: mc_create fails
    with a message instead of running a wrong transform."""
    import marlcov
    from marlcov import _lib
    g = np.ones((1090, 40))
    with pytest.raises(_lib.MarlcovError, match="extended rows exceed"):
        marlcov.BatchCoverageEnv(base_cfg(numrobot=2, dist_reward=1), 1, grids=[g], seed=1)
