"""Import alias for the framework package.

The package directory is ``cuda-mpi-gpu-cluster-programming_amd/`` (a name that is not a valid
Python identifier); ``import anx`` binds it as the ``anx`` package so every submodule resolves
as ``anx.<name>`` (``anx.ops``, ``anx.models``, ``anx.parallel`` ...).
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "cuda-mpi-gpu-cluster-programming_amd")
_spec = _ilu.spec_from_file_location("anx", _os.path.join(_dir, "__init__.py"), submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["anx"] = _mod
_spec.loader.exec_module(_mod)

if __name__ == "__main__":  # ``python -m anx <command>`` from the repo root
    from anx.__main__ import main as _main

    _main()
