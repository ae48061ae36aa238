"""Python side of the native shared-memory request/response channels (``csrc/host/shm_channel.cpp``).

``ShmServer(n_slots, slot_bytes)`` creates a uniquely named POSIX shm segment; each env worker attaches
``ShmClient(name, slot, tag)`` to its own slot.  Requests are read by the server in place (a read-only
memoryview into shared memory: no pipe copies), responses are written back into the slot, and both
sides block on futexes.  The extension is host-only C++ (``applestar_amd/_host*.so``); it is built by
``python -m applestar_amd.csrc.build`` (``build_host``) and loaded on demand.
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys
import uuid

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_mod = None


def native():
    """The ``_host`` extension module (raises with a build hint when it is missing)."""
    global _mod
    if _mod is None:
        override = os.environ.get('APPLESTAR_HOST_EXT_PATH')  # sanitizer variants
        cands = [override] if override else sorted(glob.glob(os.path.join(_PKG, '_host*.so')))
        if not cands:
            raise RuntimeError('applestar_amd host runtime not built; run `python -m applestar_amd.csrc.build`')
        spec = importlib.util.spec_from_file_location('applestar_amd._host', cands[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules['applestar_amd._host'] = mod
        _mod = mod
    return _mod


def available() -> bool:
    try:
        native()
        return True
    except (RuntimeError, OSError, ImportError):
        return False


def new_name(prefix: str = 'applestar') -> str:
    return f'/{prefix}_{os.getpid()}_{uuid.uuid4().hex[:12]}'


def ShmServer(n_slots: int, slot_bytes: int, name: str | None = None):
    return native().ShmServer(name or new_name(), int(n_slots), int(slot_bytes))


def ShmClient(name: str, slot: int, tag: int = 0):
    return native().ShmClient(name, int(slot), int(tag))
