"""Thin Python wrappers (autograd Functions) around the HIP kernels in ``applestar_amd/_C``."""
from __future__ import annotations

from . import _ext

_HAS = set()


def ensure_loaded():
    mod = _ext.require()
    if not _HAS:
        _HAS.update(n for n in dir(mod) if not n.startswith('_'))
    return mod


def has(name: str) -> bool:
    return name in _HAS and name in globals()
