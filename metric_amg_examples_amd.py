"""Import shim: the package directory is ``metric-amg-examples_amd/`` (a name
Python cannot import directly).  ``import metric_amg_examples_amd`` from the
repo root loads it as a regular package under this importable name."""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), 'metric-amg-examples_amd')
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_PKG_DIR, '__init__.py'),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
