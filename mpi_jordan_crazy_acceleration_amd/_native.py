"""Loader of the in-tree native module ``_C`` (HIP kernels + C++ engine + RCCL communicator).

The module is built by ``make`` (or ``__graft_entry__.build()``) into this directory.  It shares the
HIP runtime and RCCL that torch already loaded, so torch is imported first.  There is no Python or
eager-PyTorch fallback for the solver: if the extension is missing the import fails loudly.
"""
from __future__ import annotations

import importlib
import os

from .runtime_env import configure_runtime_env

configure_runtime_env()  # before anything initialises HIP (runtime_env.py)

import torch  # noqa: E402,F401  -- must be loaded before _C (shared libamdhip64 / librccl)

_C = None


def load_native():
    global _C
    if _C is None:
        try:
            _C = importlib.import_module(__package__ + "._C")
        except ImportError as e:  # pragma: no cover - exercised only on a broken build
            here = os.path.dirname(os.path.abspath(__file__))
            raise ImportError(
                "native extension mpi_jordan_crazy_acceleration_amd._C is not built "
                f"(looked in {here}); run `make -j` in the repository root or "
                "`python -c 'import __graft_entry__ as g; g.build()'`"
            ) from e
    return _C


def native_available() -> bool:
    try:
        load_native()
        return True
    except ImportError:
        return False


def native_path() -> str:
    return load_native().__file__
