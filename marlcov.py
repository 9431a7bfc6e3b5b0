"""Import shim: the package directory is ``marl-coverage_amd/`` (not a Python
identifier), so ``import marlcov`` loads it by path as ``marl_coverage_amd``."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "marl-coverage_amd")
if "marl_coverage_amd" not in _sys.modules:
    _spec = _ilu.spec_from_file_location("marl_coverage_amd", _os.path.join(_PKG_DIR, "__init__.py"),
                                         submodule_search_locations=[_PKG_DIR])
    _mod = _ilu.module_from_spec(_spec)
    _sys.modules["marl_coverage_amd"] = _mod
    _spec.loader.exec_module(_mod)
_sys.modules[__name__] = _sys.modules["marl_coverage_amd"]
