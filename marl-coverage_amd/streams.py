"""Host restatement of the device random streams (NumPy, vectorised).

Every random draw on the device is Philox4x32-10 keyed by a seed and a
counter that holds the GLOBAL env / grid id (mc_config env_offset /
grid_offset).  These functions reproduce those draws on the
host bit for bit, so a caller can know without a device round trip which grid
``mc_generate_grids`` made, which start cells a reset draws and which actions
``mc_random_actions`` writes — and tests can check the device against them.

    philox4x32_10        csrc/mc_device.h philox()
    generated_grid       csrc/mc_grid_kernels.hip gen_grids_kernel
    start_cells          csrc/mc_env_kernel.hip reset_env (rejection draw,
                         acceptance rule of dec_grid_rl.py:491-502)
    random_actions       csrc/mc_grid_kernels.hip random_actions_kernel
"""
from __future__ import annotations

import numpy as np

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)

# counter tags (the fourth counter word) of the device streams
TAG_PLACE = 0x706C6163  # "plac": start-cell candidates
TAG_GRID = 0x67726964   # "grid": reset_grid_mode="random" grid pick
TAG_GEN = 0x67656E21    # "gen!": synthetic grid pool
TAG_ACTS = 0x61637473   # "acts": synthetic actions


def philox4x32_10(seed: int, c0, c1, c2, c3):
    """Philox4x32-10 (Salmon et al., SC'11) of counters (c0, c1, c2, c3)
    (broadcastable uint32 arrays) under the 64-bit key ``seed``; returns the
    four uint32 output words."""
    c = [np.asarray(x, dtype=np.uint64) & _MASK for x in np.broadcast_arrays(c0, c1, c2, c3)]
    k0, k1 = int(seed) & 0xFFFFFFFF, (int(seed) >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + _W0) & 0xFFFFFFFF
        k1 = (k1 + _W1) & 0xFFFFFFFF
    return [x.astype(np.uint32) for x in c]


def bounded(r, n: int):
    """floor(r * n / 2^32): the device's uniform draw in [0, n)."""
    return ((np.asarray(r, dtype=np.uint64) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


def obstacle_threshold(p_obst: float) -> int:
    """mc_generate_grids' 32-bit threshold (launch_gen): obstacle iff r < t."""
    t = p_obst * 4294967296.0
    return 0xFFFFFFFF if t >= 4294967295.0 else (0 if t <= 0.0 else int(t))


def generated_grid(seed: int, p_obst: float, width: int, length: int, grid_id: int) -> np.ndarray:
    """The PADDED float64 grid (+1 free, -1 obstacle and border) that
    mc_generate_grids makes for global grid ``grid_id`` (width/length are the
    padded sizes): cell (x, y) is an obstacle iff word (y & 7) & 3 of
    Philox(seed, (grid_id, x, 2*(y >> 3) + ((y & 7) >> 2), TAG_GEN)) is below
    the threshold."""
    x = np.arange(width)[:, None]
    y = np.arange(length)[None, :]
    words = philox4x32_10(seed, grid_id, x, 2 * (y >> 3) + ((y & 7) >> 2), TAG_GEN)
    t = (y & 7) & 3
    r = np.select([t == 0, t == 1, t == 2, t == 3], words)
    obst = r < obstacle_threshold(p_obst) if p_obst > 0.0 else np.zeros(r.shape, bool)
    border = (x == 0) | (x == width - 1) | (y == 0) | (y == length - 1)
    return np.where(obst | border, -1.0, 1.0)


def start_cells(seed: int, env_id: int, episode: int, padded_grid, num_agents: int,
                max_candidates: int = 1 << 20) -> np.ndarray:
    """Start cells [N, 2] of the device's rejection draw for global env
    ``env_id`` at its ``episode``-th reset (1 = the first): candidate k is
    (bounded(r.x, Wp), bounded(r.y, Lp)) of Philox(seed, (k, env_id, episode,
    TAG_PLACE)), accepted iff grid >= 0 and not already taken, in order of k
    (dec_grid_rl.py:491-502)."""
    g = np.asarray(padded_grid)
    Wp, Lp = g.shape
    out, taken = [], set()
    k0, chunk = 0, 256
    while len(out) < num_agents and k0 < max_candidates:
        k = np.arange(k0, k0 + chunk, dtype=np.uint64)
        r = philox4x32_10(seed, k, env_id, episode, TAG_PLACE)
        cx, cy = bounded(r[0], Wp), bounded(r[1], Lp)
        for x, y in zip(cx.tolist(), cy.tolist()):
            if g[x, y] >= 0 and (x, y) not in taken:
                taken.add((x, y))
                out.append((x, y))
                if len(out) == num_agents:
                    break
        k0 += chunk
    if len(out) < num_agents:
        raise RuntimeError("could not place every robot (device: ERR_PLACEMENT)")
    return np.asarray(out, dtype=np.int32)


def random_actions(seed: int, env_ids, step: int, num_agents: int) -> np.ndarray:
    """uint8 [len(env_ids), N] of mc_random_actions: agent i of env e at step t
    is bits 2i, 2i+1 of word i // 16 of Philox(seed, (e, t, 0, TAG_ACTS))."""
    e = np.asarray(env_ids, dtype=np.uint64)
    w = np.stack(philox4x32_10(seed, e, step, 0, TAG_ACTS), axis=-1)  # [n, 4]
    i = np.arange(num_agents)
    return ((w[:, i >> 4] >> (2 * (i & 15)).astype(np.uint32)) & 3).astype(np.uint8)
