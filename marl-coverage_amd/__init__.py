"""marl-coverage_amd — MI355X-native batched multi-agent grid-coverage environment.

Drop-in for the env hot path of ExistentialRobotics/MARL-Coverage
(``Environments/dec_grid_rl.py:DecGridRL``): the step/reset path runs as
hand-written HIP kernels for gfx950 in ``libmarlcov.so`` (csrc/), bound through
the C ABI of ``include/marlcov.h`` with ctypes.  Import it as ``marlcov``
(the repo-root shim ``marlcov.py``) or by path.
"""
from .sensors import LidarSensor, SquareSensor, beam_angles, beam_increments  # noqa: F401
from .gridmaker import gridgen, gridload  # noqa: F401
from .action_spaces import Continuous, Discrete  # noqa: F401


def __getattr__(name):
    # the env classes need the HIP library: import lazily so that config /
    # grid helpers stay usable (and testable) on a host without it
    if name in ("BatchCoverageEnv", "pad_grid", "grid_to_int8"):
        from . import batch_env
        return getattr(batch_env, name)
    if name in ("DecGridRL", "decode_action"):
        from . import dec_grid_rl
        return getattr(dec_grid_rl, name)
    if name == "episodes":
        from . import episodes
        return episodes
    if name in ("SuperGridRL", "BatchSuperGridEnv", "decode_super_action"):
        from . import super_env
        return getattr(super_env, name)
    raise AttributeError(name)
