"""Grid sources of the reference (``Utils/gridmaker.py``).

``gridgen`` draws Bernoulli obstacle grids with NumPy's global RNG in the same
call sequence as the reference, so seeded pools are identical.  ``gridload``
reads PNG maps (black = -1 obstacle, ``clip(img - 1, -1, 1)``) or, with no
config, returns the reference's nine hand-made 15x15 grids, shipped as data
(``data/handmade15.npz``, captured from the reference by
tests/golden/make_golden.py).
"""
from __future__ import annotations

import os

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "handmade15.npz")


def gridgen(grid_config):
    """``gridmaker.py:107-139`` including its split quirk: with more than one
    grid the test set is empty (``gridlis[l:]`` with ``l = len(gridlis)``)."""
    p = grid_config["prob_obst"]
    w, l = grid_config["gridwidth"], grid_config["gridlen"]
    grids = [np.random.choice(a=[1.0, -1.0], size=(w, l), p=[1 - p, p])
             for _ in range(grid_config["numgrids"])]
    n = len(grids)
    if n == 1:
        return grids, grids
    return grids[:n], grids[n:]


def gridload(grid_config=None, sort=False):
    """``gridmaker.py:7-104``.  ``sort=True`` orders PNG files by name instead
    of the filesystem's ``os.listdir`` order the reference uses."""
    if grid_config is None:
        z = np.load(_DATA, allow_pickle=False)
        return [g.astype(np.float64) for g in z["train"]], [g.astype(np.float64) for g in z["test"]]
    from PIL import Image

    grid_dir, limit = grid_config["grid_dir"], grid_config["numgrids"]
    names = os.listdir(grid_dir)
    if sort:
        names = sorted(names)
    grids = []
    for i, fname in enumerate(names):
        if i < limit:
            img = np.array(Image.open(os.path.join(grid_dir, fname))).astype(float)
            grids.append(np.clip(img - 1, -1, 1))
    half = len(grids) // 2
    if half == 1:
        return grids, grids
    return grids[:half], grids[half:]
