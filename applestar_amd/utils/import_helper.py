"""Optional-dependency probes (``distar/ctools/utils/import_helper.py:8-120``).

Each ``try_import_*`` returns the module (or the reference's tuple) when importable and ``None``
otherwise, warning once.  ``try_import_link`` returns ``torch.distributed`` — the reference's
"linklink" collective library is replaced by torch.distributed over RCCL here, and the reference's
``FakeLink`` fallback corresponds to :mod:`applestar_amd.parallel.dist` running single-process.
"""
from __future__ import annotations

import importlib
import warnings
from typing import List

_warned = set()


def _missing(name: str):
    if name not in _warned:
        warnings.warn(f'optional package {name!r} is not installed')
        _warned.add(name)


def try_import_redis():
    try:
        import redis  # noqa: F401
        from redis.client import StrictRedis
        return redis, StrictRedis
    except ImportError:
        _missing('redis')
        return None, None


def try_import_ceph():
    try:
        import ceph  # noqa: F401
        return ceph
    except ImportError:
        _missing('ceph')
        return None


def try_import_mc():
    try:
        import mc  # noqa: F401
        return mc
    except ImportError:
        _missing('mc')
        return None


def try_import_link():
    import torch.distributed as dist
    return dist


def import_module(modules: List[str]) -> None:
    """Import every module path in ``modules`` (plugin registration side effects)."""
    for m in modules:
        importlib.import_module(m)
