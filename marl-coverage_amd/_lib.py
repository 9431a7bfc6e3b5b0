"""ctypes binding of libmarlcov.so (include/marlcov.h).

There is no CPU fallback: if the HIP library is missing or does not export the
ABI this package expects, importing the env classes raises.  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (or ``build.py``).
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmarlcov.so")
ABI_VERSION = 9

MC_OK, MC_EINVAL, MC_EHIP, MC_ESTATE, MC_EDEVICE = 0, -1, -2, -3, -4
SENSOR_LIDAR, SENSOR_SQUARE = 0, 1
PARAM_DIST_CACHE_CELLS, PARAM_DIST_T, PARAM_DIST_MAX_ROWS = 0, 1, 2  # mc_build_param
ACT_SENTINEL = 255
ACT_NOOP = 4

(FIELD_POS, FIELD_MOVED, FIELD_FREE, FIELD_OBST, FIELD_VISITED, FIELD_FREE_COUNT,
 FIELD_VISITED_COUNT, FIELD_CURRSTEP, FIELD_DONE_THRESH, FIELD_ENV_GRID, FIELD_EPISODE,
 FIELD_NUMFREE, FIELD_GRID_NEG, FIELD_GRID_POS, FIELD_DIST_MW, FIELD_DIST_LISTED, FIELD_EP_PC,
 FIELD_EP_LEN, FIELD_DJ_LISTED, FIELD_DIST_CACHED, FIELD_DIST_TOTALS) = range(21)


class McConfig(ctypes.Structure):
    """Mirror of ``mc_config`` (include/marlcov.h)."""

    _fields_ = [
        ("num_envs", ctypes.c_int32),
        ("num_agents", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("length", ctypes.c_int32),
        ("num_grids", ctypes.c_int32),
        ("sensor_type", ctypes.c_int32),
        ("num_beams", ctypes.c_int32),
        ("square_radius", ctypes.c_int32),
        ("lidar_range", ctypes.c_double),
        ("egoradius", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("collision_penalty", ctypes.c_double),
        ("terminal_reward", ctypes.c_double),
        ("done_thresh", ctypes.c_double),
        ("done_incr", ctypes.c_double),
        ("maxsteps", ctypes.c_int32),
        ("comm_radius", ctypes.c_int32),
        ("map_sharing", ctypes.c_int32),
        ("single_square_tool", ctypes.c_int32),
        ("dist_reward", ctypes.c_int32),
        ("dijkstra_input", ctypes.c_int32),
        ("auto_reset", ctypes.c_int32),
        ("reset_grid_mode", ctypes.c_int32),
        ("mini_map_rad", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("env_offset", ctypes.c_uint32),
        ("grid_offset", ctypes.c_uint32),
    ]


class McLayout(ctypes.Structure):
    """Mirror of ``mc_layout``."""

    _fields_ = [
        ("tile_rows", ctypes.c_int32),
        ("tile_cols", ctypes.c_int32),
        ("window_half", ctypes.c_int32),
        ("window_tiles", ctypes.c_int32),
        ("obs_layers", ctypes.c_int32),
        ("obs_side", ctypes.c_int32),
        ("obs_bytes_per_env", ctypes.c_int64),
        ("mask_words_per_agent", ctypes.c_int64),
        ("state_bytes", ctypes.c_int64),
    ]


class McSgConfig(ctypes.Structure):
    """Mirror of ``mc_sg_config`` (SuperGridRL handles)."""

    _fields_ = [
        ("num_envs", ctypes.c_int32),
        ("num_agents", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("length", ctypes.c_int32),
        ("num_grids", ctypes.c_int32),
        ("senseradius", ctypes.c_int32),
        ("collision_penalty", ctypes.c_double),
        ("free_penalty", ctypes.c_double),
        ("terminal_reward", ctypes.c_double),
        ("done_thresh", ctypes.c_double),
        ("done_incr", ctypes.c_double),
        ("dist_reward", ctypes.c_int32),
        ("use_scanning", ctypes.c_int32),
        ("maxsteps", ctypes.c_int32),
        ("auto_reset", ctypes.c_int32),
        ("reset_grid_mode", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("env_offset", ctypes.c_uint32),
        ("grid_offset", ctypes.c_uint32),
    ]


class McSgLayout(ctypes.Structure):
    """Mirror of ``mc_sg_layout``."""

    _fields_ = [
        ("pos_layers", ctypes.c_int32),
        ("obs_layers", ctypes.c_int32),
        ("row_words", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("state_bytes", ctypes.c_int64),
    ]


(SG_FIELD_POS, SG_FIELD_COVERED, SG_FIELD_OBST, SG_FIELD_COV_COUNT, SG_FIELD_CURRSTEP,
 SG_FIELD_DONE_THRESH, SG_FIELD_A_PREV, SG_FIELD_ENV_GRID, SG_FIELD_EPISODE, SG_FIELD_NUMPOS,
 SG_FIELD_GRID_NEG, SG_FIELD_GRID_POS, SG_FIELD_EP_PC, SG_FIELD_EP_LEN) = range(14)


# (name, restype, argtypes) for every symbol include/marlcov.h declares
_VP, _I32, _I64, _U64, _D = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
SIGNATURES = [
    ("mc_abi_version", _I32, []),
    ("mc_last_error", ctypes.c_char_p, []),
    ("mc_struct_size", _I64, [_I32]),
    ("mc_build_param", _I64, [_I32]),
    ("mc_create", ctypes.c_int, [ctypes.POINTER(McConfig), ctypes.c_int, ctypes.POINTER(_VP)]),
    ("mc_destroy", None, [_VP]),
    ("mc_query", ctypes.c_int, [_VP, ctypes.POINTER(McLayout)]),
    ("mc_set_beam_table", ctypes.c_int, [_VP, _VP, _I32]),
    ("mc_set_grids", ctypes.c_int, [_VP, _VP, _I32, _VP]),
    ("mc_generate_grids", ctypes.c_int, [_VP, _U64, _D, _VP]),
    ("mc_set_env_grids", ctypes.c_int, [_VP, _VP, _VP]),
    ("mc_random_actions", ctypes.c_int, [_VP, _U64, _I32, _VP, _VP]),
    ("mc_kernel_variant", ctypes.c_char_p, [_VP]),
    ("mc_reset", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    ("mc_step", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("mc_step_many", ctypes.c_int, [_VP, _VP, _I64, _I32, _VP, _I64, _VP, _I64, _VP, _I64, _VP, _I64, _VP]),
    ("mc_field_bytes", _I64, [_VP, _I32]),
    ("mc_get_state", ctypes.c_int, [_VP, _I32, _VP, _I64, _VP]),
    ("mc_set_state", ctypes.c_int, [_VP, _I32, _VP, _I64, _VP]),
    ("mc_check", ctypes.c_int, [_VP, _VP]),
    ("mc_debug_stamps", ctypes.c_int, [_VP, _VP]),
    ("mc_set_dist_obs", ctypes.c_int, [_VP, _VP]),
    ("mc_set_minimap_obs", ctypes.c_int, [_VP, _VP]),
    ("mc_sg_create", ctypes.c_int, [ctypes.POINTER(McSgConfig), ctypes.c_int, ctypes.POINTER(_VP)]),
    ("mc_sg_destroy", None, [_VP]),
    ("mc_sg_query", ctypes.c_int, [_VP, ctypes.POINTER(McSgLayout)]),
    ("mc_sg_set_grids", ctypes.c_int, [_VP, _VP, _I32, _VP]),
    ("mc_sg_generate_grids", ctypes.c_int, [_VP, _U64, _D, _VP]),
    ("mc_sg_set_env_grids", ctypes.c_int, [_VP, _VP, _VP]),
    ("mc_sg_set_obs", ctypes.c_int, [_VP, _VP, _VP]),
    ("mc_sg_reset", ctypes.c_int, [_VP, _VP, _VP, _VP]),
    ("mc_sg_step", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    ("mc_sg_field_bytes", _I64, [_VP, _I32]),
    ("mc_sg_get_state", ctypes.c_int, [_VP, _I32, _VP, _I64, _VP]),
    ("mc_sg_set_state", ctypes.c_int, [_VP, _I32, _VP, _I64, _VP]),
    ("mc_sg_check", ctypes.c_int, [_VP, _VP]),
]

_lib = None


class MarlcovError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load and type the library once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("MARLCOV_LIB", LIB_PATH)
    if not os.path.exists(path):
        raise ImportError(
            f"libmarlcov.so not found at {path}: the HIP extension is required "
            "(there is no CPU fallback). Build it with __graft_entry__.build().")
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mc_abi_version() != ABI_VERSION:
        raise ImportError(f"libmarlcov ABI {lib.mc_abi_version()} != expected {ABI_VERSION}")
    mirrors = (McConfig, McLayout, McSgConfig, McSgLayout)
    if any(lib.mc_struct_size(i) != ctypes.sizeof(m) for i, m in enumerate(mirrors)):
        raise ImportError("libmarlcov struct layout mismatch (mc_config / mc_layout / mc_sg_*)")
    _lib = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != MC_OK:
        msg = _lib.mc_last_error().decode(errors="replace") if _lib is not None else ""
        raise MarlcovError(f"{what} failed ({rc}): {msg}")
    return rc
