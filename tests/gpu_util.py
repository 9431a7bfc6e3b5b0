"""Helpers shared by the GPU parity tests: unpack device bit masks, build an
oracle env from device state, compare device env <-> oracle env."""
from __future__ import annotations

import numpy as np

from oracle.cpu_ref import DecGridRLRef


def unpack_tiles(tiles, rows, cols):
    """int64 [..., TR, TC] 8x8-cell tiles -> uint8 [..., rows, cols] cells."""
    from marlcov.tiles import tiles_to_cells
    return tiles_to_cells(tiles, rows, cols)


def device_state(env, envs=None):
    """Host copies of every per-env state field of a BatchCoverageEnv.  With
    ``envs`` (a list of env indices) the bit maps are unpacked only for those
    envs (and their grids) and come back as dicts keyed by env / grid index:
    C5-sized batches would otherwise unpack gigabytes per step."""
    from marlcov import _lib
    W, L = env.width, env.length

    def get(f):
        return env.get_state(f).cpu().numpy()

    st = {
        "pos": get(_lib.FIELD_POS),
        "moved": get(_lib.FIELD_MOVED).astype(np.uint64),
        "free_cnt": get(_lib.FIELD_FREE_COUNT),
        "vis_cnt": get(_lib.FIELD_VISITED_COUNT),
        "currstep": get(_lib.FIELD_CURRSTEP),
        "done_thresh": get(_lib.FIELD_DONE_THRESH),
        "env_grid": get(_lib.FIELD_ENV_GRID),
        "episode": get(_lib.FIELD_EPISODE),
        "numfree": get(_lib.FIELD_NUMFREE),
    }
    maps = {"free": _lib.FIELD_FREE, "obst": _lib.FIELD_OBST, "vis": _lib.FIELD_VISITED}
    grids = {"neg": _lib.FIELD_GRID_NEG, "pos_plane": _lib.FIELD_GRID_POS}
    if envs is None:
        for k, f in {**maps, **grids}.items():
            st[k] = unpack_tiles(get(f), W, L)
        return st
    envs = [int(b) for b in envs]
    gids = sorted({int(st["env_grid"][b]) for b in envs})
    for k, f in maps.items():
        t = env.get_state(f)
        sel = unpack_tiles(t[envs].cpu().numpy(), W, L)
        st[k] = {b: sel[i] for i, b in enumerate(envs)}
    for k, f in grids.items():
        t = env.get_state(f)
        sel = unpack_tiles(t[gids].cpu().numpy(), W, L)
        st[k] = {g: sel[i] for i, g in enumerate(gids)}
    return st


def compare_env(st, b, ref, tag=""):
    """Device state of env b vs oracle env ``ref`` (bit-exact)."""
    p = ref._pad
    W, L = ref._gridwidth, ref._gridlen
    np.testing.assert_array_equal(st["pos"][b, :, 0], ref._xinds, err_msg=tag + " x")
    np.testing.assert_array_equal(st["pos"][b, :, 1], ref._yinds, err_msg=tag + " y")
    rf = (ref._free_pad[:, p:p + W, p:p + L] > 0).astype(np.uint8)
    ro = (ref._obst_pad[:, p:p + W, p:p + L] > 0).astype(np.uint8)
    np.testing.assert_array_equal(st["free"][b], rf, err_msg=tag + " free")
    np.testing.assert_array_equal(st["obst"][b], ro, err_msg=tag + " obst")
    np.testing.assert_array_equal(st["vis"][b], (ref._visited > 0).astype(np.uint8), err_msg=tag + " vis")
    assert int(st["free_cnt"][b]) == np.count_nonzero(ref._free_pad > 0), tag
    assert int(st["vis_cnt"][b]) == int(np.sum(ref._visited)), tag
    assert int(st["currstep"][b]) == ref._currstep, tag
    assert float(st["done_thresh"][b]) == float(ref._done_thresh), tag
    moved = int(st["moved"][b])
    rp = np.zeros((W + 2 * p, L + 2 * p))
    for i in range(ref._numrobot):
        if (moved >> i) & 1:
            rp[ref._xinds[i] + p, ref._yinds[i] + p] = 1
    np.testing.assert_array_equal(rp, ref._robot_pad, err_msg=tag + " robot_pad")


def oracle_from_device(st, b, env_config, thetalist=None):
    """Build a DecGridRLRef holding exactly the device state of env b."""
    g = st["env_grid"][b]
    grid = np.where(st["neg"][g] == 1, -1.0, np.where(st["pos_plane"][g] == 1, 1.0, 0.0))
    inner = grid[1:-1, 1:-1]
    np.random.seed(0)
    ref = DecGridRLRef([inner], env_config)
    if thetalist is not None:
        ref._sensor.set_thetalist(thetalist)
    p = ref._pad
    W, L = grid.shape
    N = ref._numrobot
    ref._grid = grid
    ref._xinds = st["pos"][b, :, 0].astype(int).copy()
    ref._yinds = st["pos"][b, :, 1].astype(int).copy()
    ref._robot_pos_map = np.zeros((W, L))
    ref._robot_pos_map[ref._xinds, ref._yinds] = 1
    ref._robot_pad = np.zeros((W + 2 * p, L + 2 * p))
    moved = int(st["moved"][b])
    for i in range(N):
        if (moved >> i) & 1:
            ref._robot_pad[ref._xinds[i] + p, ref._yinds[i] + p] = 1
    ref._free_pad = np.zeros((N, W + 2 * p, L + 2 * p))
    ref._obst_pad = np.zeros((N, W + 2 * p, L + 2 * p))
    ref._free_pad[:, p:p + W, p:p + L] = st["free"][b]
    ref._obst_pad[:, p:p + W, p:p + L] = st["obst"][b]
    ref._visited = st["vis"][b].astype(np.float64)
    ref._currstep = int(st["currstep"][b])
    ref._done_thresh = float(st["done_thresh"][b])
    ref._numfree = int(np.count_nonzero(grid > 0))
    ref.updateCommmunicationGraph()
    return ref


def ref_action(codes_row):
    """uint8 per-agent codes -> the oracle's action (None = sentinel)."""
    if codes_row[0] == 255:
        return None
    return np.asarray(codes_row, dtype=np.int64)
