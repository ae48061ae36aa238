"""Safe, zero-copy serialisation of tensor trees (trajectories, model weights) for the data plane.

The reference pickles trajectories and models and lz4-compresses them (``file_helper.py:255-302``);
unpickling untrusted bytes executes code and every tensor is copied several times.  Here a tree of
dict/list/tuple/tensor/number/str/None is encoded as

    magic | u64 header_len | JSON header (tree with tensor descriptors) | padding | raw tensor bytes

Each tensor's bytes are 64-byte aligned, so the receiver can ``torch.frombuffer`` the payload in
place — e.g. straight out of a pinned receive buffer — and issue one ``hipMemcpyAsync`` per batch.
Optional zlib compression (lz4 is not available on these images) is applied to the whole frame.

Uncompressed frames are encoded / decoded by the native codec (``csrc/codec.cpp``, same format) when the
extension is importable: a tensor leaf costs a type check and a memcpy instead of ~10 us of Python attribute
calls (an agent-step request is ~120 leaves, a trajectory ~10k).  ``APPLESTAR_NATIVE_CODEC=0`` forces the
Python codec (both are tested against each other).
"""
from __future__ import annotations

import io
import json
import os
import struct
import zlib
from typing import Any, List, Tuple

import numpy as np
import torch

MAGIC = b'ASTR1'
_ALIGN = 64

_DT = {torch.float32: 'f32', torch.float16: 'f16', torch.bfloat16: 'bf16', torch.float64: 'f64',
       torch.int64: 'i64', torch.int32: 'i32', torch.int16: 'i16', torch.int8: 'i8', torch.uint8: 'u8',
       torch.bool: 'b'}
_DT_INV = {v: k for k, v in _DT.items()}


def _encode(obj: Any, blobs: List[torch.Tensor], offset: List[int]):
    if torch.is_tensor(obj):
        t = obj.detach()
        if t.device.type != 'cpu':
            t = t.cpu()
        t = t.contiguous()
        off = (offset[0] + _ALIGN - 1) // _ALIGN * _ALIGN
        nbytes = t.numel() * t.element_size()
        blobs.append((off, t))
        offset[0] = off + nbytes
        return {'__t__': [_DT[t.dtype], list(t.shape), off, nbytes]}
    if isinstance(obj, dict):
        return {'__d__': [[k, _encode(v, blobs, offset)] for k, v in obj.items()]}
    if isinstance(obj, (list, tuple)):
        return {'__l__' if isinstance(obj, list) else '__tu__': [_encode(v, blobs, offset) for v in obj]}
    if isinstance(obj, np.ndarray):
        return _encode(torch.from_numpy(np.ascontiguousarray(obj)), blobs, offset)
    if obj is None or isinstance(obj, (bool, int, float, str)):
        return {'__v__': obj}
    if isinstance(obj, (np.integer, np.floating)):
        return {'__v__': obj.item()}
    raise TypeError(f'cannot serialise {type(obj)}')


_NATIVE = None


def _native():
    global _NATIVE
    if _NATIVE is None:
        _NATIVE = False
        if os.environ.get('APPLESTAR_NATIVE_CODEC', '1') != '0':
            try:
                from ..ops import _ext
                mod = _ext._load()
                if mod is not None and hasattr(mod, 'tree_dumps'):
                    _NATIVE = mod
            except Exception:  # pragma: no cover - extension missing / broken: Python codec
                _NATIVE = False
    return _NATIVE


def dumps(tree: Any, compress: bool = False) -> bytes:
    if not compress:
        nat = _native()
        if nat:
            try:
                return nat.tree_dumps(tree)
            except TypeError:     # numpy leaves and other types the native encoder leaves to Python
                pass
    return dumps_py(tree, compress)


def dumps_py(tree: Any, compress: bool = False) -> bytes:
    blobs: List[Tuple[int, torch.Tensor]] = []
    offset = [0]
    header = json.dumps(_encode(tree, blobs, offset)).encode()
    body = bytearray(offset[0])
    dst = np.frombuffer(body, dtype=np.uint8)
    for off, t in blobs:
        if t.numel():
            flat = t.reshape(-1)
            raw = flat.view(torch.uint8) if t.dtype != torch.bool else flat.to(torch.uint8)
            dst[off:off + raw.numel()] = raw.numpy()
    pre = MAGIC + struct.pack('<QB', len(header), 1 if compress else 0)
    pad = (-(len(pre) + len(header))) % _ALIGN
    frame = bytes(pre) + header + b'\0' * pad
    data = bytes(body)
    if compress:
        data = zlib.compress(data, 1)
    return frame + data


def _decode(node: Any, buf: memoryview, copy: bool):
    if '__t__' in node:
        dt, shape, off, nbytes = node['__t__']
        dtype = _DT_INV[dt]
        if nbytes == 0:
            return torch.empty(shape, dtype=dtype)
        base = torch.bool if dtype == torch.bool else dtype
        load_dt = torch.uint8 if dtype == torch.bool else base
        t = torch.frombuffer(buf, dtype=load_dt, count=nbytes // torch.empty(0, dtype=load_dt).element_size(),
                             offset=off).view(shape)
        if dtype == torch.bool:
            t = t.to(torch.bool)
        return t.clone() if copy else t
    if '__d__' in node:
        return {k: _decode(v, buf, copy) for k, v in node['__d__']}
    if '__l__' in node:
        return [_decode(v, buf, copy) for v in node['__l__']]
    if '__tu__' in node:
        return tuple(_decode(v, buf, copy) for v in node['__tu__'])
    return node['__v__']


def loads(data, copy: bool = True) -> Any:
    """Decode a frame.  ``copy=False`` returns tensors aliasing ``data`` (must stay alive/writable)."""
    nat = _native()
    if nat and len(data) > len(MAGIC) + 8 and memoryview(data)[len(MAGIC) + 8] == 0:
        return nat.tree_loads(data, copy)
    return loads_py(data, copy)


def loads_py(data, copy: bool = True) -> Any:
    mv = memoryview(data)
    if bytes(mv[:len(MAGIC)]) != MAGIC:
        raise ValueError('not an applestar frame')
    hlen, comp = struct.unpack('<QB', mv[len(MAGIC):len(MAGIC) + 9])
    hstart = len(MAGIC) + 9
    header = json.loads(bytes(mv[hstart:hstart + hlen]))
    body_start = hstart + hlen + ((-(hstart + hlen)) % _ALIGN)
    body = mv[body_start:]
    if comp:
        body = memoryview(bytearray(zlib.decompress(body)))
        copy = False if not copy else copy
    elif not copy:
        body = body  # aliasing view
    else:
        body = memoryview(bytearray(body))
        copy = False  # already a private buffer
    return _decode(header, body, copy)


def parse(data):
    """(header tree, body memoryview) of an uncompressed frame without decoding any tensor; tensor
    leaves stay ``{'__t__': [dtype, shape, body_offset, nbytes]}`` descriptors (trajectory ring)."""
    mv = memoryview(data)
    if bytes(mv[:len(MAGIC)]) != MAGIC:
        raise ValueError('not an applestar frame')
    hlen, comp = struct.unpack('<QB', mv[len(MAGIC):len(MAGIC) + 9])
    if comp:
        raise ValueError('compressed frames cannot be parsed in place')
    hstart = len(MAGIC) + 9
    header = json.loads(bytes(mv[hstart:hstart + hlen]))
    body_start = hstart + hlen + ((-(hstart + hlen)) % _ALIGN)
    return header, mv[body_start:]


DTYPES = _DT_INV


def save(tree: Any, path: str, compress: bool = False) -> None:
    with open(path, 'wb') as f:
        f.write(dumps(tree, compress))


def load(path: str) -> Any:
    with open(path, 'rb') as f:
        return loads(f.read())
