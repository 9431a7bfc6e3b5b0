"""Import shim: the package directory is ``marl-coverage_amd/`` (not a Python
identifier), so ``import marlcov`` loads it by path as ``marl_coverage_amd``.
Submodules imported as ``marlcov.<name>`` are the SAME module objects as
``marl_coverage_amd.<name>`` (a meta-path alias), so classes compare equal
whichever name imported them."""
import importlib
import importlib.abc
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


class _Alias(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    """marlcov.<sub> -> the already-loaded (or freshly imported) marl_coverage_amd.<sub>."""

    def find_spec(self, name, path=None, target=None):
        if name.startswith("marlcov."):
            return _ilu.spec_from_loader(name, self)
        return None

    def create_module(self, spec):
        return importlib.import_module("marl_coverage_amd" + spec.name[len("marlcov"):])

    def exec_module(self, module):
        pass


if not any(isinstance(f, _Alias) for f in _sys.meta_path):
    _sys.meta_path.insert(0, _Alias())
_sys.modules[__name__] = _sys.modules["marl_coverage_amd"]
