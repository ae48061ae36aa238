"""File / payload helpers with the reference's ``fs_type`` surface (``ctools/utils/file_helper.py``).

``dumps(data, fs_type, compress)`` / ``loads(bytes, fs_type, compress)``:

* ``'applestar'`` (default) -- :mod:`serialize` frames (JSON header + aligned raw tensor bytes, safe);
* ``'torch'`` -- ``torch.save`` bytes; loaded with ``weights_only=True`` (tensors/containers only);
* ``'numpy'`` (alias ``'nppickle'``/``'npcPickle'``) -- a nested tree whose arrays are stored as ``.npy``
  members of an in-memory npz with a JSON structure file (``allow_pickle=False`` on load);
* ``'pickle'``/``'cPickle'`` -- refused unless ``allow_pickle=True`` is passed explicitly: unpickling
  executes code, so it is only for bytes this process wrote itself.

``compress`` applies zlib level 1 (lz4 is not available on these images).  ``read_file`` /
``save_file`` / ``remove_file`` mirror the reference's path helpers (local filesystem; the
ceph/memcached back-ends are disabled in the reference too); ``save_traj_file``/``load_traj_file`` keep
trajectories in the safe frame format.
"""
from __future__ import annotations

import io
import json
import os
import pickle
import zlib
from typing import Any

import numpy as np
import torch

from . import serialize
from .checkpoint import load_file, save_file as _save_torch

_NP_ALIASES = ('numpy', 'nppickle', 'npcPickle')
_PICKLE = ('pickle', 'cPickle')


def _np_encode(obj, arrays):
    if torch.is_tensor(obj):
        obj = obj.detach().cpu().numpy()
    if isinstance(obj, np.ndarray):
        arrays.append(obj)
        return {'__nd__': len(arrays) - 1}
    if isinstance(obj, dict):
        return {'__d__': [[k, _np_encode(v, arrays)] for k, v in obj.items()]}
    if isinstance(obj, (list, tuple)):
        return {'__l__' if isinstance(obj, list) else '__t__': [_np_encode(v, arrays) for v in obj]}
    if isinstance(obj, np.generic):
        return obj.item()
    return obj


def _np_decode(node, arrays):
    if isinstance(node, dict):
        if '__nd__' in node:
            return arrays[node['__nd__']]
        if '__d__' in node:
            return {k: _np_decode(v, arrays) for k, v in node['__d__']}
        if '__l__' in node:
            return [_np_decode(v, arrays) for v in node['__l__']]
        if '__t__' in node:
            return tuple(_np_decode(v, arrays) for v in node['__t__'])
    return node


def dumps(data: Any, fs_type: str = 'applestar', compress: bool = False) -> bytes:
    if fs_type == 'applestar':
        return serialize.dumps(data, compress=compress)
    if fs_type == 'torch':
        buf = io.BytesIO()
        torch.save(data, buf)
        raw = buf.getvalue()
    elif fs_type in _NP_ALIASES:
        arrays = []
        tree = _np_encode(data, arrays)
        buf = io.BytesIO()
        np.savez(buf, __tree__=np.frombuffer(json.dumps(tree).encode(), dtype=np.uint8),
                 **{f'a{i}': a for i, a in enumerate(arrays)})
        raw = buf.getvalue()
    elif fs_type in _PICKLE:
        raw = pickle.dumps(data, protocol=pickle.HIGHEST_PROTOCOL)
    else:
        raise ValueError(f'unknown fs_type {fs_type!r}')
    return zlib.compress(raw, 1) if compress else raw


def loads(data: bytes, fs_type: str = 'applestar', compress: bool = False, allow_pickle: bool = False) -> Any:
    if fs_type == 'applestar':
        return serialize.loads(data)
    raw = zlib.decompress(data) if compress else bytes(data)
    if fs_type == 'torch':
        return torch.load(io.BytesIO(raw), map_location='cpu', weights_only=True)
    if fs_type in _NP_ALIASES:
        with np.load(io.BytesIO(raw), allow_pickle=False) as z:
            tree = json.loads(bytes(z['__tree__']).decode())
            arrays = [z[f'a{i}'] for i in range(len(z.files) - 1)]
        return _np_decode(tree, arrays)
    if fs_type in _PICKLE:
        if not allow_pickle:
            raise PermissionError('pickle payloads execute code on load; pass allow_pickle=True only for '
                                  'bytes this process produced')
        return pickle.loads(raw)
    raise ValueError(f'unknown fs_type {fs_type!r}')


def read_file(path: str, fs_type: str = 'torch') -> Any:
    """``fs_type`` 'torch' -> ``torch.load(weights_only=True)``; 'applestar'/'numpy' -> safe frames."""
    if fs_type == 'torch':
        return load_file(path)
    with open(path, 'rb') as f:
        return loads(f.read(), fs_type)


def save_file(path: str, data: Any, fs_type: str = 'torch') -> None:
    """Atomic write (temp file + rename)."""
    if fs_type == 'torch':
        _save_torch(data, path)
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + '.tmp'
    with open(tmp, 'wb') as f:
        f.write(dumps(data, fs_type))
    os.replace(tmp, path)


def remove_file(path: str, fs_type: str = 'normal') -> None:
    if os.path.exists(path):
        os.remove(path)


def save_traj_file(data: Any, path: str, fs_type: str = 'applestar') -> None:
    save_file(path, data, fs_type)


def load_traj_file(path: str, fs_type: str = 'applestar') -> Any:
    return read_file(path, fs_type)
