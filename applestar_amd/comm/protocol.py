"""Tensor wire codec of the coordinator data plane (``distar/ctools/worker/coordinator/protocol.py:17-85``:
``encode`` / ``decode`` of nested tensor structures).  Here both are the zero-copy, pickle-free frame
format of :mod:`applestar_amd.utils.serialize` (64-B aligned tensor payloads after a JSON header), so a
receiver can view tensors in place from a pinned buffer."""
from __future__ import annotations

from typing import Any

from ..utils import serialize


def encode(data: Any, compress: bool = False) -> bytes:
    return serialize.dumps(data, compress=compress)


def decode(buf) -> Any:
    return serialize.loads(buf)
