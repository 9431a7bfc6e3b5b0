"""CPU-only tests: the C-ABI library loads and exports every symbol of
include/marlcov.h (no compute calls without a GPU), config validation, and
the host-side logic of the package (action decoding, beam table, grids)."""
import ctypes
import os
import re

import numpy as np
import pytest

from golden_util import GOLDEN_DIR, load_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    import marlcov
    from marlcov import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _lib.load()


def header_functions():
    src = open(os.path.join(ROOT, "include", "marlcov.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mc_[a-z_]+)\s*\(", src)))


def test_header_symbols_exported_and_typed(lib):
    from marlcov import _lib
    names = header_functions()
    assert len(names) >= 15
    typed = {n for n, _, _ in _lib.SIGNATURES}
    for n in names:
        assert hasattr(lib, n), f"{n} not exported"
        assert n in typed, f"{n} has no ctypes signature"


def test_struct_layout_and_version(lib):
    from marlcov import _lib
    assert lib.mc_abi_version() == _lib.ABI_VERSION
    assert lib.mc_struct_size(0) == ctypes.sizeof(_lib.McConfig)
    assert lib.mc_struct_size(1) == ctypes.sizeof(_lib.McLayout)
    assert lib.mc_struct_size(2) == ctypes.sizeof(_lib.McSgConfig)
    assert lib.mc_struct_size(3) == ctypes.sizeof(_lib.McSgLayout)
    assert lib.mc_struct_size(7) == -1


def test_build_params(lib):
    """mc_build_param: the distance transform's build constants (kDistK,
    kDistT, the row limit) that bench.py prices C5 with."""
    from marlcov import _lib
    assert lib.mc_build_param(_lib.PARAM_DIST_CACHE_CELLS) == 512
    assert lib.mc_build_param(_lib.PARAM_DIST_T) == 20
    # the distance transform's row limit: the big-map kernel past the LDS
    # bitboard's 832 rows (bg2_1073x1073: 1,079 extended rows at egoradius 2)
    assert lib.mc_build_param(_lib.PARAM_DIST_MAX_ROWS) == 1088
    assert lib.mc_build_param(99) == -1


def _cfg(**kw):
    from marlcov import _lib
    c = _lib.McConfig()
    c.num_envs, c.num_agents, c.width, c.length, c.num_grids = 4, 4, 130, 130, 4
    c.sensor_type, c.num_beams, c.lidar_range = _lib.SENSOR_LIDAR, 21, 10.0
    c.egoradius, c.pad = 2, 2
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("bad,msg", [
    (dict(num_envs=0), "num_envs"),
    (dict(num_agents=65), "numrobot"),
    (dict(num_agents=0), "numrobot"),
    (dict(width=2), "padded grid"),
    (dict(lidar_range=40.0), "range"),
    (dict(egoradius=40, pad=40), "egoradius"),
    (dict(num_agents=64, sensor_type=1, square_radius=20), "window tiles"),
    (dict(sensor_type=7), "sensor_type"),
    (dict(pad=1), "pad"),
])
def test_create_rejects_bad_config(lib, bad, msg):
    h = ctypes.c_void_p()
    rc = lib.mc_create(ctypes.byref(_cfg(**bad)), 0, ctypes.byref(h))
    assert rc == -1 and not h.value
    assert msg in lib.mc_last_error().decode()


def test_null_arguments_are_errors(lib):
    assert lib.mc_create(None, 0, None) == -1
    assert lib.mc_step(None, None, None, None, None, None, None) == -1
    assert lib.mc_step_many(None, None, 0, 1, None, 0, None, 0, None, 0, None, 0, None) == -1
    assert lib.mc_reset(None, None, None, None, None, None) == -1
    assert lib.mc_query(None, None) == -1


def test_decode_action_reference_semantics():
    from marlcov.dec_grid_rl import decode_action
    assert decode_action(None, 3) is None
    assert decode_action(-1, 3) is None
    assert decode_action(np.array([-1]), 1) is None
    assert list(decode_action(27, 3)) == [3, 2, 1]             # base 4, robot 0 = LSD
    assert list(decode_action(-2, 2)) == [2, 3]                # Python floor semantics
    assert list(decode_action(np.int64(6), 2)) == [2, 1]
    assert list(decode_action(2.5, 1)) == [4]                  # not 0..3 -> no-op
    assert list(decode_action(np.array([7]), 1)) == [4]
    assert list(decode_action([0, 3, 9], 3)) == [0, 3, 4]      # per-agent superset
    assert list(decode_action(4 ** 16 - 1, 16)) == [3] * 16


def test_beam_table_matches_golden_bits():
    from marlcov import beam_angles, beam_increments
    z = np.load(os.path.join(GOLDEN_DIR, "beam_tables.npz"))
    for key in z.files:
        tab = beam_increments(beam_angles(int(key[1:])))
        np.testing.assert_array_equal(tab.view(np.uint64), z[key].view(np.uint64), err_msg=key)


def test_gridload_handmade_matches_reference():
    from marlcov import gridload
    train, test = gridload(None)
    case = load_case("square_r2_single_tool_handmade")
    assert len(train) == 6 and len(test) == 3
    np.testing.assert_array_equal(np.stack(train), case["train"].astype(np.float64))
    np.testing.assert_array_equal(np.stack(test), case["test"].astype(np.float64))


def test_gridgen_rng_sequence_and_split():
    from marlcov import gridgen
    np.random.seed(4)
    tr, te = gridgen(dict(prob_obst=0.2, gridwidth=9, gridlen=7, numgrids=3))
    np.random.seed(4)
    exp = [np.random.choice(a=[1.0, -1.0], size=(9, 7), p=[0.8, 0.2]) for _ in range(3)]
    assert te == [] and len(tr) == 3
    for a, b in zip(tr, exp):
        np.testing.assert_array_equal(a, b)
    tr, te = gridgen(dict(prob_obst=0.2, gridwidth=9, gridlen=7, numgrids=1))
    assert tr is te


def test_grid_values_validated():
    from marlcov.batch_env import grid_to_int8, pad_grid
    g = pad_grid(np.array([[1.0, 0.0], [-1.0, 1.0]]))
    assert g.shape == (4, 4) and g[0, 0] == -1
    np.testing.assert_array_equal(grid_to_int8(g)[1:3, 1:3], [[1, 0], [-1, 1]])
    with pytest.raises(ValueError):
        grid_to_int8(np.array([[0.5]]))


def test_bench_bytes_formula_matches_survey():
    import bench
    assert bench.algorithmic_bytes_per_env_step(1, 10, 2) == 893
    assert bench.algorithmic_bytes_per_env_step(4, 10, 2) == 3476
    assert bench.algorithmic_bytes_per_env_step(8, 20, 2) == 24280
    # C5: SURVEY 8(d)'s figure (a full-map read per agent and step) ...
    assert bench.algorithmic_bytes_per_env_step(16, 10, 2, layers=7, full_map_cells=518 ** 2) == 1088720


def test_c5_design_bytes_formula():
    """The C5 bench line's roofline bytes: the windowed 8(d)
    part, 16 x (441 + 336 + 175 + 9) + 32 = 15,408 B per env-step, plus per
    step the maps fully transformed (ceil(518^2 / 8) = 33,541 B bit-map read
    + 4,128 B cache write), the maps the cache served (4,128 B cache read) and
    4 B per listed map, from the MC_FIELD_DIST_TOTALS deltas."""
    import bench
    f = bench.c5_design_bytes_per_step
    assert f(1, 16, 10, 2, 518, 0, 0, 0, 1) == 15408
    assert bench.dist_cache_bytes() == 4128  # kDistK from the library (mc_build_param)
    # 100 listed over 2 launches: 60 served, 40 full transforms
    extra = 40 * (33541 + 4128) + 60 * 4128 + 100 * 4
    assert f(8192, 16, 10, 2, 518, 100, 60, 40, 2) == 8192 * 15408 + extra / 2


def test_tile_block_layout_round_trip():
    """marlcov.tiles mirrors the device map order (include/marlcov.h, ABI v3):
    4x4 blocks of 8x8-cell tiles, tile_index = ((ti/4)*TCS + tj/4)*16 +
    (ti%4)*4 + tj%4, bit 8*r + c = cell (8*ti + r, 8*tj + c)."""
    import numpy as np
    from marlcov.tiles import blocks_to_tiles, cells_to_tiles, tiles_to_cells
    rng = np.random.default_rng(3)
    cells = (rng.random((2, 3, 130, 70)) < 0.3).astype(np.uint8)
    blocks = cells_to_tiles(cells, blocks=True)
    assert blocks.shape == (2, 3, 5, 3, 4, 4) and blocks.dtype == np.uint64
    np.testing.assert_array_equal(tiles_to_cells(blocks, 130, 70), cells)
    grid = blocks_to_tiles(blocks)
    flat = blocks.reshape(2, 3, -1)
    tcs = blocks.shape[3]
    for ti, tj in [(0, 0), (5, 7), (16, 8), (13, 3)]:
        idx = ((ti >> 2) * tcs + (tj >> 2)) * 16 + (ti & 3) * 4 + (tj & 3)
        assert flat[1, 2, idx] == grid[1, 2, ti, tj]
        r, c = 3, 6
        bit = (int(grid[1, 2, ti, tj]) >> (8 * r + c)) & 1
        x, y = 8 * ti + r, 8 * tj + c
        assert bit == (cells[1, 2, x, y] if x < 130 and y < 70 else 0)


def test_super_action_decode_reference_semantics():
    """super_grid_rl.py:88-98,203-208: base-4 digits slot 0 first, the quotient
    is what motion_penalty sees (KeyError unless 0 <= q < 4), -1/None sentinel."""
    from marlcov.super_env import decode_super_action
    assert decode_super_action(None, 2) is None
    assert decode_super_action(-1, 3) is None
    d, q = decode_super_action(4 * 3 + 2, 2)
    assert d.tolist() == [2, 3] and q == 0
    d, q = decode_super_action(3 * 16 + 7, 2)
    assert d.tolist() == [3, 1] and q == 3
    with pytest.raises(KeyError):
        decode_super_action(4 * 16, 2)
    with pytest.raises(KeyError):
        decode_super_action(-2, 1)
    d, q = decode_super_action(np.int64(9), 2)
    assert d.tolist() == [1, 2] and q == 0
    d, q = decode_super_action([1, 7, 3], 3)
    assert d.tolist() == [1, 4, 3] and q == 0


def test_super_row_bitboards_round_trip():
    from marlcov.super_env import pack_rows, unpack_rows
    rs = np.random.RandomState(0)
    for shape in [(3, 1), (5, 63), (4, 64), (7, 65), (2, 130)]:
        c = (rs.rand(2, *shape) < 0.4).astype(np.uint8)
        w = pack_rows(c)
        assert w.shape == (2, shape[0], (shape[1] + 63) // 64)
        np.testing.assert_array_equal(unpack_rows(w, shape[1]), c)
        # bit (y & 63) of word y >> 6 is cell y (include/marlcov.h)
        x, y = 1, shape[1] - 1
        assert ((int(w[0, x, y >> 6]) >> (y & 63)) & 1) == c[0, x, y]


def test_super_create_rejects_bad_config(lib):
    from marlcov import _lib
    c = _lib.McSgConfig(num_envs=1, num_agents=2, width=8, length=8, num_grids=1, senseradius=1)
    h = ctypes.c_void_p()
    for field, bad in (("num_agents", 65), ("senseradius", 16), ("width", 0), ("num_envs", 0)):
        cc = _lib.McSgConfig.from_buffer_copy(c)
        setattr(cc, field, bad)
        assert lib.mc_sg_create(ctypes.byref(cc), 0, ctypes.byref(h)) == _lib.MC_EINVAL
        assert lib.mc_last_error()


def test_gridload_png_semantics(tmp_path):
    """Utils/gridmaker.py:82-104: PNG maps -> clip(img - 1, -1, 1) as float64,
    at most numgrids files in os.listdir order, half/half split with the
    len // 2 == 1 quirk (both sets = every map; one map: empty train set)."""
    from PIL import Image
    from marlcov import gridload
    rs = np.random.RandomState(3)
    imgs = {}
    for i in range(5):
        img = rs.choice(np.array([0, 1, 2, 255], dtype=np.uint8), size=(9, 11))
        name = f"map{i}.png"
        Image.fromarray(img, mode="L").save(tmp_path / name)
        imgs[name] = np.clip(img.astype(float) - 1, -1, 1)
    cfg = {"grid_dir": str(tmp_path), "numgrids": 4}
    train, test = gridload(cfg, sort=True)
    names = sorted(imgs)[:4]
    assert len(train) == 2 and len(test) == 2
    for g, n in zip(train + test, names):
        assert g.dtype == np.float64 and set(np.unique(g)) <= {-1.0, 0.0, 1.0}
        np.testing.assert_array_equal(g, imgs[n])
    tr, te = gridload({"grid_dir": str(tmp_path), "numgrids": 3}, sort=True)
    assert len(tr) == 3 and len(te) == 3          # 3 // 2 == 1: both sets are every map
    tr, te = gridload({"grid_dir": str(tmp_path), "numgrids": 1}, sort=True)
    assert len(tr) == 0 and len(te) == 1          # 1 // 2 == 0: the reference's empty train set
    tr, te = gridload({"grid_dir": str(tmp_path), "numgrids": 10})  # filesystem order, all 5
    assert len(tr) == 2 and len(te) == 3


def test_episode_config_cut():
    """marlcov.episodes.episode_config folds generate_episode's cut
    (utils.py:25-28: _currstep == test/train maxsteps) into the env's maxsteps
    (DecGridRL.done, dec_grid_rl.py:544): the smaller one ends the episode."""
    from marlcov.episodes import episode_config
    c = dict(maxsteps=1000, train_maxsteps=300, test_maxsteps=50)
    assert episode_config(c, testing=True)["maxsteps"] == 50
    assert episode_config(c, testing=False)["maxsteps"] == 300
    c = dict(maxsteps=20, train_maxsteps=300, test_maxsteps=50)
    assert episode_config(c, testing=True)["maxsteps"] == 20
    assert c["maxsteps"] == 20  # the caller's dict is not modified


def test_sensor_listeners_are_weak():
    """A sensor shared by several device envs holds them weakly (a dropped
    env is not kept alive and is skipped on set_thetalist)."""
    import gc

    from marlcov.sensors import LidarSensor
    calls = []

    class Holder:
        def upload(self, sensor):
            calls.append(sensor._num_lasers)

    s = LidarSensor({"num_lasers": 5, "range": 3})
    a, b = Holder(), Holder()
    s.add_listener(a.upload)
    s.add_listener(b.upload)
    s.set_thetalist(np.linspace(0, 2 * np.pi, 7, endpoint=False))
    assert calls == [7, 7]
    del a
    gc.collect()
    s.set_thetalist(np.linspace(0, 2 * np.pi, 9, endpoint=False))
    assert calls == [7, 7, 9] and len(s._listeners) == 1
    s.remove_listener(b.upload)
    s.set_thetalist(np.linspace(0, 2 * np.pi, 3, endpoint=False))
    assert calls == [7, 7, 9] and s._listeners == []


def test_philox_known_answers():
    """marlcov.streams restates the device's Philox4x32-10 (csrc/mc_device.h):
    pinned to the Random123 known-answer vectors (kat_vectors, philox4x32_10)."""
    from marlcov.streams import philox4x32_10
    kat = [
        ((0, 0, 0, 0), 0, (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, 0xFFFFFFFFFFFFFFFF, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), 0x299F31D0A4093822,
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in kat:
        got = tuple(int(x) for x in philox4x32_10(key, *ctr))
        assert got == want, (ctr, [hex(x) for x in got])


def test_host_streams_shapes_and_rules():
    """Host mirrors of the device streams: the gen grid has the -1 border and
    about p_obst obstacles; start cells are distinct free cells; actions are
    0..3 and depend only on (global env id, step)."""
    from marlcov.streams import generated_grid, random_actions, start_cells
    g = generated_grid(1000, 0.1, 130, 130, 7)
    assert g.shape == (130, 130) and set(np.unique(g)) <= {-1.0, 1.0}
    assert np.all(g[0] == -1) and np.all(g[-1] == -1) and np.all(g[:, 0] == -1) and np.all(g[:, -1] == -1)
    frac = np.mean(g[1:-1, 1:-1] < 0)
    assert 0.08 < frac < 0.12
    assert not np.array_equal(g, generated_grid(1000, 0.1, 130, 130, 8))
    cells = start_cells(1, 7, 1, g, 4)
    assert len({tuple(c) for c in cells}) == 4 and all(g[x, y] >= 0 for x, y in cells)
    a = random_actions(12345, [3, 4, 5], 9, 16)
    assert a.shape == (3, 16) and a.max() <= 3
    np.testing.assert_array_equal(a[1:], random_actions(12345, [4, 5], 9, 16))
    assert not np.array_equal(a, random_actions(12345, [3, 4, 5], 10, 16))


def test_kernel_variant_null_env(lib):
    assert lib.mc_kernel_variant(None) == b""
    assert "null" in lib.mc_last_error().decode()
    assert lib.mc_random_actions(None, 0, 0, None, None) == -1


def test_gridload_reference_png_maps(tmp_path):
    """marlcov.gridload on the reference's own PNG maps (Grids/bg2_100x100,
    bg2_1073x1073; copies in tests/golden/maps): the grids equal what the
    reference's gridload produced from the same files
    (tests/golden/bg2_100x100_stc.npz, gridmaker.py:82-102), values in
    {-1, 1} from mode-L {0, 255} pixels, the train / test split of two files
    (train = test = both, :96-98), and sort=True orders by file name."""
    import shutil

    import marlcov
    maps = os.path.join(os.path.dirname(__file__), "golden", "maps")
    for n in os.listdir(maps):
        if n.startswith("bg2_100x100__"):
            shutil.copyfile(os.path.join(maps, n), tmp_path / n.split("__", 1)[1])
    train, test = marlcov.gridload({"grid_dir": str(tmp_path), "numgrids": 30}, sort=True)
    assert len(train) == len(test) == 2
    assert all(a is b for a, b in zip(train, test))
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "bg2_100x100_stc.npz"))
    assert sorted(g.astype(np.int8).tobytes() for g in train) == sorted(g.tobytes() for g in z["test_grids"])
    big = tmp_path / "big"
    big.mkdir()
    shutil.copyfile(os.path.join(maps, "bg2_1073x1073__AR0011SR.png"), big / "AR0011SR.png")
    train, test = marlcov.gridload({"grid_dir": str(big), "numgrids": 30})
    assert train == [] and len(test) == 1 and test[0].shape == (1073, 1073)
    assert set(np.unique(test[0]).tolist()) <= {-1.0, 1.0}
