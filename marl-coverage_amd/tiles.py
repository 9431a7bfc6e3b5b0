"""Host conversion of the device's tiled bit maps (include/marlcov.h).

A map is uint64 [..., tile_rows/4, tile_cols/4, 4, 4]: 4x4 blocks of 8x8-cell
tiles (one 128-byte line per block); bit 8*r + c of tile (ti, tj) is cell
(8*ti + r, 8*tj + c), and tile (ti, tj) sits at block (ti//4, tj//4), slot
(ti%4, tj%4).  These helpers are plumbing for state inspection (the
reference's _free_pad / _obst_pad / _visited arrays), not the hot path.
"""
from __future__ import annotations

import numpy as np


def blocks_to_tiles(blocks) -> np.ndarray:
    """[..., TRS, TCS, 4, 4] block order -> [..., 4*TRS, 4*TCS] tile grid."""
    b = np.asarray(blocks)
    lead, (trs, tcs) = b.shape[:-4], b.shape[-4:-2]
    return np.moveaxis(b, -2, -3).reshape(lead + (4 * trs, 4 * tcs))


def tiles_to_blocks(tiles) -> np.ndarray:
    """[..., TR, TC] tile grid (TR, TC multiples of 4) -> [..., TR/4, TC/4, 4, 4]."""
    t = np.asarray(tiles)
    lead, (tr, tc) = t.shape[:-2], t.shape[-2:]
    return np.ascontiguousarray(np.moveaxis(t.reshape(lead + (tr // 4, 4, tc // 4, 4)), -3, -2))


def tiles_to_cells(tiles, rows: int, cols: int) -> np.ndarray:
    """uint64/int64 tiles -> uint8 [..., rows, cols] cells.  Accepts the device
    block order [..., TRS, TCS, 4, 4] or a plain tile grid [..., TR, TC]."""
    t = np.asarray(tiles)
    if t.ndim >= 4 and t.shape[-2:] == (4, 4):
        t = blocks_to_tiles(t)
    t = np.ascontiguousarray(t).astype(np.uint64)
    lead, (tr, tc) = t.shape[:-2], t.shape[-2:]
    b = np.unpackbits(t.view(np.uint8).reshape(t.shape + (8,)), axis=-1, bitorder="little")
    b = b.reshape(lead + (tr, tc, 8, 8))            # [..., ti, tj, r, c]
    b = np.moveaxis(b, -2, -3)                      # [..., ti, r, tj, c]
    return b.reshape(lead + (tr * 8, tc * 8))[..., :rows, :cols]


def cells_to_tiles(cells, blocks: bool = False) -> np.ndarray:
    """uint8/bool [..., rows, cols] cells -> uint64 tiles: a plain grid
    [..., TR, TC] (TR = ceil(rows/8) rounded up to a multiple of 4, likewise TC),
    or with blocks=True the device order [..., TR/4, TC/4, 4, 4]."""
    c = np.asarray(cells) != 0
    lead, (rows, cols) = c.shape[:-2], c.shape[-2:]
    tr, tc = -(-rows // 32) * 4, -(-cols // 32) * 4
    full = np.zeros(lead + (tr * 8, tc * 8), dtype=np.uint8)
    full[..., :rows, :cols] = c
    b = full.reshape(lead + (tr, 8, tc, 8))
    b = np.moveaxis(b, -3, -2)                      # [..., ti, tj, r, c]
    packed = np.packbits(b.reshape(lead + (tr, tc, 64)), axis=-1, bitorder="little")
    grid = np.ascontiguousarray(packed).view(np.uint64).reshape(lead + (tr, tc))
    return tiles_to_blocks(grid) if blocks else grid
