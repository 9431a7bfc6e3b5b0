"""Host conversion of the device's 8x8-cell tiled bit maps (include/marlcov.h).

A map is uint64 [..., tile_rows, tile_cols]; bit 8*r + c of tile (ti, tj) is
cell (8*ti + r, 8*tj + c).  These helpers are plumbing for state inspection
(the reference's _free_pad / _obst_pad / _visited arrays), not the hot path.
"""
from __future__ import annotations

import numpy as np


def tiles_to_cells(tiles, rows: int, cols: int) -> np.ndarray:
    """uint64/int64 [..., TR, TC] tiles -> uint8 [..., rows, cols] cells."""
    t = np.ascontiguousarray(np.asarray(tiles)).astype(np.uint64)
    lead, (tr, tc) = t.shape[:-2], t.shape[-2:]
    b = np.unpackbits(t.view(np.uint8).reshape(t.shape + (8,)), axis=-1, bitorder="little")
    b = b.reshape(lead + (tr, tc, 8, 8))            # [..., ti, tj, r, c]
    b = np.moveaxis(b, -2, -3)                      # [..., ti, r, tj, c]
    return b.reshape(lead + (tr * 8, tc * 8))[..., :rows, :cols]


def cells_to_tiles(cells) -> np.ndarray:
    """uint8/bool [..., rows, cols] cells -> uint64 [..., ceil(rows/8), ceil(cols/8)]."""
    c = np.asarray(cells) != 0
    lead, (rows, cols) = c.shape[:-2], c.shape[-2:]
    tr, tc = -(-rows // 8), -(-cols // 8)
    full = np.zeros(lead + (tr * 8, tc * 8), dtype=np.uint8)
    full[..., :rows, :cols] = c
    b = full.reshape(lead + (tr, 8, tc, 8))
    b = np.moveaxis(b, -3, -2)                      # [..., ti, tj, r, c]
    packed = np.packbits(b.reshape(lead + (tr, tc, 64)), axis=-1, bitorder="little")
    return np.ascontiguousarray(packed).view(np.uint64).reshape(lead + (tr, tc))
