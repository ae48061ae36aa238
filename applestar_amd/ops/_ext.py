"""Loader for the in-tree HIP extension ``applestar_amd/_C*.so`` (built by
``applestar_amd/csrc/build.py`` for gfx950).

Policy: tensors on a GPU must run the native kernels.  If the extension is missing on a machine
that has a GPU we raise (``require()``) instead of silently falling back to PyTorch; CPU tensors run
the PyTorch reference implementations in :mod:`applestar_amd.ops.reference` (CPU-only play and the
CPU test-suite).
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_C = None
_ERR: str | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    override = os.environ.get('APPLESTAR_EXT_PATH')  # debug / host-sanitizer build variants
    cands = [override] if override else sorted(glob.glob(os.path.join(_PKG_DIR, '_C*.so')))
    if not cands:
        _ERR = f'applestar_amd native extension not built (no _C*.so in {_PKG_DIR}); run `python -m applestar_amd.csrc.build`'
        return None
    try:
        import torch  # noqa: F401  (extension links against libtorch / c10_hip)
        spec = importlib.util.spec_from_file_location('applestar_amd._C', cands[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules['applestar_amd._C'] = mod
        _C = mod
    except Exception as e:  # pragma: no cover - depends on the machine
        _ERR = f'failed to load {cands[0]}: {e!r}'
    return _C


def available() -> bool:
    return _load() is not None


def require():
    mod = _load()
    if mod is None:
        raise RuntimeError(_ERR)
    return mod


def error() -> str | None:
    _load()
    return _ERR
