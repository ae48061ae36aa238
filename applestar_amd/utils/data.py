"""Nested-structure data helpers: device/dtype/tensor conversion, collate / decollate, list<->dict
transposes, locks and small defaults (``distar/ctools/utils/{data_helper,default_helper,lock_helper}.py``,
``ctools/torch_utils/{data_helper,detach}.py``, ``ctools/data/collate_fn.py``).

The learner's hot collate path does not use these (trajectories are assembled on the GPU from the
HBM ring, :mod:`applestar_amd.runtime.traj_ring`); they serve tools, SL/replay utilities and plugins.
:class:`DevicePrefetcher` is the ``CudaFetcher`` equivalent: it stages the next batch to the GPU on a
side HIP stream while the current one is consumed.
"""
from __future__ import annotations

import collections.abc as cabc
import functools
import logging
import multiprocessing
import queue
import re
import threading
from enum import Enum
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional, Sequence

import numpy as np
import torch

_np_str = re.compile(r'[SaUO]')


# ---------------------------------------------------------------------------------------------- conversion
def to_device(item: Any, device, ignore_keys: Sequence[str] = (), non_blocking: bool = False) -> Any:
    if torch.is_tensor(item) or isinstance(item, torch.nn.Module):
        return item.to(device, non_blocking=non_blocking) if torch.is_tensor(item) else item.to(device)
    if isinstance(item, Mapping):
        return {k: (v if k in ignore_keys else to_device(v, device, ignore_keys, non_blocking))
                for k, v in item.items()}
    if isinstance(item, tuple) and hasattr(item, '_fields'):
        return type(item)(*[to_device(v, device, ignore_keys, non_blocking) for v in item])
    if isinstance(item, (list, tuple)):
        return type(item)(to_device(v, device, ignore_keys, non_blocking) for v in item)
    return item


def to_dtype(item: Any, dtype: torch.dtype) -> Any:
    if torch.is_tensor(item):
        return item.to(dtype)
    if isinstance(item, Mapping):
        return {k: to_dtype(v, dtype) for k, v in item.items()}
    if isinstance(item, (list, tuple)):
        return type(item)(to_dtype(v, dtype) for v in item)
    raise TypeError(f'to_dtype: unsupported {type(item)}')


def to_tensor(item: Any, dtype: Optional[torch.dtype] = None, ignore_keys: Sequence[str] = (),
              transform_scalar: bool = True) -> Any:
    """numpy arrays / scalars / nested containers -> tensors (strings and None pass through)."""
    if item is None or isinstance(item, str):
        return item
    if torch.is_tensor(item):
        return item if dtype is None else item.to(dtype)
    if isinstance(item, np.ndarray):
        if _np_str.search(item.dtype.str):
            return item
        t = torch.from_numpy(np.ascontiguousarray(item))
        return t if dtype is None else t.to(dtype)
    if isinstance(item, (bool, int, float, np.generic)):
        if not transform_scalar:
            return item
        return torch.as_tensor(item, dtype=dtype)
    if isinstance(item, Mapping):
        return {k: (v if k in ignore_keys else to_tensor(v, dtype, ignore_keys, transform_scalar))
                for k, v in item.items()}
    if isinstance(item, tuple) and hasattr(item, '_fields'):
        return type(item)(*[to_tensor(v, dtype, ignore_keys, transform_scalar) for v in item])
    if isinstance(item, (list, tuple)):
        if item and all(isinstance(x, (int, float, bool)) for x in item):
            return torch.as_tensor(item, dtype=dtype)
        return type(item)(to_tensor(v, dtype, ignore_keys, transform_scalar) for v in item)
    raise TypeError(f'to_tensor: unsupported {type(item)}')


def to_ndarray(item: Any, dtype: Optional[np.dtype] = None) -> Any:
    if item is None or isinstance(item, str):
        return item
    if torch.is_tensor(item):
        a = item.detach().cpu().numpy()
        return a if dtype is None else a.astype(dtype)
    if isinstance(item, np.ndarray):
        return item if dtype is None else item.astype(dtype)
    if isinstance(item, (bool, int, float, np.generic)):
        return np.asarray(item, dtype=dtype)
    if isinstance(item, Mapping):
        return {k: to_ndarray(v, dtype) for k, v in item.items()}
    if isinstance(item, (list, tuple)):
        return type(item)(to_ndarray(v, dtype) for v in item)
    raise TypeError(f'to_ndarray: unsupported {type(item)}')


def tensor_to_list(item: Any) -> Any:
    if item is None:
        return None
    if torch.is_tensor(item):
        return item.tolist()
    if isinstance(item, Mapping):
        return {k: tensor_to_list(v) for k, v in item.items()}
    if isinstance(item, (list, tuple)):
        return [tensor_to_list(v) for v in item]
    if isinstance(item, (int, float, bool, np.generic)):
        return item
    raise TypeError(f'tensor_to_list: unsupported {type(item)}')


def same_shape(data: Sequence[torch.Tensor]) -> bool:
    assert isinstance(data, (list, tuple))
    return len({tuple(d.shape) for d in data}) <= 1


def get_tensor_data(data: Any) -> Any:
    """Detached copies (tensor.data) of every tensor in a nested structure."""
    if torch.is_tensor(data):
        return data.detach().clone()
    if data is None or isinstance(data, (int, float, bool, str)):
        return data
    if isinstance(data, Mapping):
        return {k: get_tensor_data(v) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return type(data)(get_tensor_data(v) for v in data)
    raise TypeError(f'get_tensor_data: unsupported {type(data)}')


def detach_grad(data: Any) -> Any:
    """In place (for containers) detach of every tensor (``torch_utils/detach.py``)."""
    if isinstance(data, list):
        for i, v in enumerate(data):
            data[i] = detach_grad(v)
    elif isinstance(data, dict):
        for k in list(data):
            data[k] = detach_grad(data[k])
    elif torch.is_tensor(data):
        data = data.detach()
    return data


# ---------------------------------------------------------------------------------------------- collate
def default_collate_with_dim(batch: Sequence, device='cpu', dim: int = 0) -> Any:
    """Stack each field of a list of samples along ``dim`` (nested dict / list / namedtuple aware)."""
    elem = batch[0]
    if torch.is_tensor(elem):
        return torch.stack(list(batch), dim=dim).to(device)
    if isinstance(elem, np.ndarray):
        if _np_str.search(elem.dtype.str):
            raise TypeError(f'cannot collate array of {elem.dtype}')
        return default_collate_with_dim([torch.as_tensor(b) for b in batch], device, dim)
    if isinstance(elem, np.generic):
        return torch.as_tensor(np.asarray(batch), device=device)
    if isinstance(elem, bool):
        return torch.tensor(batch, dtype=torch.bool, device=device)
    if isinstance(elem, (int, float)):
        return torch.tensor(batch, device=device)
    if isinstance(elem, str):
        return list(batch)
    if isinstance(elem, Mapping):
        return {k: default_collate_with_dim([d[k] for d in batch if k in d], device, dim) for k in elem}
    if isinstance(elem, tuple) and hasattr(elem, '_fields'):
        return type(elem)(*(default_collate_with_dim(s, device, dim) for s in zip(*batch)))
    if isinstance(elem, Sequence):
        if any(len(b) != len(elem) for b in batch):
            raise RuntimeError('each element in list of batch should be of equal size')
        return [default_collate_with_dim(s, device, dim) for s in zip(*batch)]
    raise TypeError(f'default_collate: unsupported {type(elem)}')


def default_collate(batch: Sequence) -> Any:
    """Stack on a new leading batch dimension; ints -> int64, floats -> float32 (reference dtypes)."""
    elem = batch[0]
    if isinstance(elem, float):
        return torch.tensor(batch, dtype=torch.float32)
    if isinstance(elem, bool):
        return torch.tensor(batch, dtype=torch.bool)
    if isinstance(elem, int):
        return torch.tensor(batch, dtype=torch.int64)
    if isinstance(elem, Mapping):
        return {k: default_collate([d[k] for d in batch]) for k in elem}
    if isinstance(elem, Sequence) and not isinstance(elem, str) and not torch.is_tensor(elem) \
            and not (isinstance(elem, tuple) and hasattr(elem, '_fields')):
        return [default_collate(s) for s in zip(*batch)]
    return default_collate_with_dim(batch)


def diff_shape_collate(batch: Sequence) -> Any:
    """Like default_collate, but tensors of different shapes stay a list and None may trail."""
    elem = batch[0]
    assert all(b is not None for b in batch[:-1]), 'None may only appear at the end of the sequence'
    if torch.is_tensor(elem):
        return torch.stack(list(batch)) if same_shape([b for b in batch if b is not None]) and batch[-1] is not None \
            else list(batch)
    if isinstance(elem, np.ndarray):
        return diff_shape_collate([torch.as_tensor(b) if b is not None else None for b in batch])
    if isinstance(elem, np.generic):
        return torch.as_tensor(np.asarray(batch))
    if isinstance(elem, bool):
        return torch.tensor(batch, dtype=torch.bool)
    if isinstance(elem, int):
        return torch.tensor(batch, dtype=torch.int64)
    if isinstance(elem, float):
        return torch.tensor(batch, dtype=torch.float32)
    if isinstance(elem, Mapping):
        return {k: diff_shape_collate([d[k] for d in batch if d is not None and k in d]) for k in elem}
    if isinstance(elem, tuple) and hasattr(elem, '_fields'):
        return type(elem)(*(diff_shape_collate(s) for s in zip(*batch)))
    if isinstance(elem, Sequence) and not isinstance(elem, str):
        return [diff_shape_collate(s) for s in zip(*batch)]
    raise TypeError(f'diff_shape_collate: unsupported {type(elem)}')


def timestep_collate(batch: List[Dict[str, Any]]) -> Dict[str, Any]:
    """[B x {key: [T x tensor]}] -> {key: tensor [T, B, ...]}, ``prev_state`` kept as a per-sample list."""
    prev = [b.pop('prev_state') for b in batch] if 'prev_state' in batch[0] else None

    def stack(x):
        if isinstance(x, Mapping):
            return {k: stack(v) for k, v in x.items()}
        if isinstance(x, (list, tuple)) and x and torch.is_tensor(x[0]):
            return torch.stack(list(x))
        return x

    out = stack(default_collate(batch))
    if prev is not None:
        out['prev_state'] = list(zip(*prev))
    return out


def default_decollate_with_dim(batch: Any, ignore: Sequence[str] = (), dim: int = 0) -> List[Any]:
    if torch.is_tensor(batch):
        return [t.squeeze(dim) for t in torch.split(batch, 1, dim=dim)]
    if isinstance(batch, Mapping):
        tmp = {k: v if k in ignore else default_decollate_with_dim(v, dim=dim) for k, v in batch.items()}
        n = len(next(iter(tmp.values())))
        return [{k: tmp[k][i] for k in tmp} for i in range(n)]
    if isinstance(batch, Sequence):
        return list(zip(*[default_decollate_with_dim(e, dim=dim) for e in batch]))
    raise TypeError(f'decollate: unsupported {type(batch)}')


def default_decollate(batch: Any, ignore: Sequence[str] = ('prev_state',)) -> List[Any]:
    """Inverse of default_collate: split the leading dimension (1-d tensors keep a [1] shape)."""
    if torch.is_tensor(batch):
        parts = list(torch.split(batch, 1, dim=0))
        return [p.squeeze(0) for p in parts] if batch.dim() > 1 else parts
    if isinstance(batch, Mapping):
        tmp = {k: v if k in ignore else default_decollate(v) for k, v in batch.items()}
        n = len(next(iter(tmp.values())))
        return [{k: tmp[k][i] for k in tmp} for i in range(n)]
    if isinstance(batch, Sequence):
        return list(zip(*[default_decollate(e) for e in batch]))
    raise TypeError(f'decollate: unsupported {type(batch)}')


# ---------------------------------------------------------------------------------------------- defaults
def lists_to_dicts(data: Sequence[Mapping], recursive: bool = False) -> Dict[Any, list]:
    """[{k: v}, ...] -> {k: [v, ...]} (optionally recursing into nested dicts)."""
    if not data:
        raise ValueError('empty input')
    if isinstance(data[0], Mapping):
        out = {k: [d[k] for d in data] for k in data[0]}
        if recursive:
            out = {k: lists_to_dicts(v, True) if isinstance(v[0], Mapping) else v for k, v in out.items()}
        return out
    if isinstance(data[0], tuple) and hasattr(data[0], '_fields'):
        return type(data[0])(*[list(x) for x in zip(*data)])
    raise TypeError(type(data[0]))


def dicts_to_lists(data: Mapping[Any, Sequence]) -> List[Dict]:
    n = len(next(iter(data.values())))
    assert all(len(v) == n for v in data.values())
    return [{k: v[i] for k, v in data.items()} for i in range(n)]


def squeeze(data: Any) -> Any:
    """Unwrap single-element lists/tuples/dicts."""
    if isinstance(data, (list, tuple)) and len(data) == 1:
        return data[0]
    if isinstance(data, dict) and len(data) == 1:
        return next(iter(data.values()))
    return data


def default_get(data: Mapping, name: str, default_value: Any = None, default_fn: Optional[Callable] = None,
                judge_fn: Optional[Callable] = None) -> Any:
    if name in data:
        return data[name]
    value = default_fn() if default_fn is not None else default_value
    if judge_fn is not None:
        assert judge_fn(value), f'default value {value!r} for {name!r} rejected'
    return value


def list_split(data: list, step: int):
    """Split into chunks of ``step``; returns (chunks, remainder or None)."""
    if len(data) < step:
        return [], data
    n = len(data) // step
    chunks = [data[i * step:(i + 1) * step] for i in range(n)]
    rest = data[n * step:]
    return chunks, (rest or None)


def override(cls: type) -> Callable:
    """Decorator asserting that the method overrides one of ``cls``."""
    def check(method):
        assert method.__name__ in dir(cls), f'{method.__name__} does not override {cls.__name__}'
        return method
    return check


def error_wrapper(fn: Callable, default_ret: Any, warning_msg: str = '[WARNING] call failed, returning default'):
    """Call ``fn`` and return ``default_ret`` (with a warning) if it raises."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        try:
            return fn(*args, **kwargs)
        except Exception as e:  # noqa: BLE001 - by contract
            logging.warning(f'{warning_msg} {type(e).__name__}: {e}')
            return default_ret
    return wrapper


class LockContextType(Enum):
    THREAD_LOCK = 1
    PROCESS_LOCK = 2


class LockContext:
    """``with LockContext(type_=...)`` over a thread or process lock."""

    def __init__(self, type_: LockContextType = LockContextType.THREAD_LOCK):
        self.lock = threading.Lock() if type_ == LockContextType.THREAD_LOCK else multiprocessing.Lock()

    def acquire(self):
        self.lock.acquire()

    def release(self):
        self.lock.release()

    def __enter__(self):
        self.lock.acquire()
        return self

    def __exit__(self, *exc):
        self.lock.release()


# ---------------------------------------------------------------------------------------------- prefetch
def _record_stream(item, stream):
    if torch.is_tensor(item):
        if item.is_cuda:
            item.record_stream(stream)
    elif isinstance(item, Mapping):
        for v in item.values():
            _record_stream(v, stream)
    elif isinstance(item, (list, tuple)):
        for v in item:
            _record_stream(v, stream)


class DevicePrefetcher:
    """Iterate a host loader while the NEXT batch is copied to ``device`` on a side stream
    (``CudaFetcher``, ``torch_utils/data_helper.py:203-232``).  Host tensors should be pinned for the
    copies to be asynchronous.  ``sleep`` / thread-based fetching is replaced by stream ordering: the
    consumer's stream waits on the copy event of the batch it receives."""

    def __init__(self, loader: Iterable, device, queue_size: int = 2):
        self.loader = iter(loader)
        self.device = torch.device(device)
        self.cuda = self.device.type == 'cuda'
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._q: 'queue.Queue' = queue.Queue(maxsize=queue_size)
        self._stop = False
        self._thread = threading.Thread(target=self._run, daemon=True, name='device-prefetch')
        self._thread.start()

    def _run(self):
        try:
            for item in self.loader:
                if self._stop:
                    break
                if self.cuda:
                    with torch.cuda.stream(self.stream):
                        dev = to_device(item, self.device, non_blocking=True)
                        ev = torch.cuda.Event()
                        ev.record(self.stream)
                else:
                    dev, ev = to_device(item, self.device), None
                self._q.put((dev, ev))
        finally:
            self._q.put(None)

    def __iter__(self):
        return self

    def __next__(self):
        got = self._q.get()
        if got is None:
            raise StopIteration
        data, ev = got
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            _record_stream(data, cur)  # the copies were allocated on the side stream
        return data

    def close(self):
        self._stop = True
