"""Host -> HBM batch staging on a side HIP stream.

The learner's next batch is copied from pinned host memory with ``non_blocking`` copies issued on a
dedicated copy stream while the current step computes (the reference does this in a separate
process with its own CUDA stream and a multiprocessing queue, ``rl_dataloader.py:113-127,160-169``).
The compute stream waits on an event recorded after the copies, and every staged tensor is marked
``record_stream`` so the caching allocator does not recycle it early.

``pin_tree`` packs a batch dict into ONE pinned byte buffer (every tensor a view of it; done once per
batch by the producer thread): staging is then one H2D copy plus cheap device views, instead of ~120
``.to(device)`` calls (each a host-side launch of ~15-25 us on the learner thread, and one or more blit
kernels on the GPU) per RL batch.
"""
from __future__ import annotations

from typing import Any, Iterator, Optional

import os

import torch

PACKED_H2D = os.environ.get('APPLESTAR_PACKED_H2D', '1') == '1'

_ALIGN = 64


class PackedBatch(dict):
    """A host batch dict whose tensors are views of one pinned uint8 buffer ``self.buffer``.
    ``self.template`` is the batch with each tensor replaced by its slot index in ``self.slots``
    ((byte offset, dtype, shape) per tensor)."""

    def __init__(self, tree, buffer, template, slots):
        super().__init__(tree)
        self.buffer, self.template, self.slots = buffer, template, slots

    def to_device(self, device, record_stream=None):
        """One non_blocking copy of the buffer; the batch rebuilt as device views of it."""
        dbuf = self.buffer.to(device, non_blocking=True)
        if record_stream is not None:
            dbuf.record_stream(record_stream)
        views = []
        for off, dtype, shape in self.slots:
            n = _nbytes(dtype, shape)
            views.append(dbuf[off:off + n].view(dtype).view(shape))
        return _fill(self.template, views)


class _Slot:
    __slots__ = ('i',)

    def __init__(self, i):
        self.i = i


def _nbytes(dtype, shape) -> int:
    n = torch.empty((), dtype=dtype).element_size()
    for d in shape:
        n *= d
    return n


def _fill(t, views):
    if isinstance(t, _Slot):
        return views[t.i]
    if isinstance(t, dict):
        return {k: _fill(v, views) for k, v in t.items()}
    if isinstance(t, list):
        return [_fill(v, views) for v in t]
    if isinstance(t, tuple):
        return tuple(_fill(v, views) for v in t)
    return t


def pack_tree(batch: dict, pin: bool = None) -> PackedBatch:
    """Copy every tensor of ``batch`` into one pinned buffer (64-byte aligned slots); the returned dict
    holds host views of it, so host-side readers (e.g. :func:`entity_total_hint`) still work."""
    tensors, slots = [], []
    off = 0

    def walk(x):
        nonlocal off
        if torch.is_tensor(x):
            x = x.detach().contiguous()
            slots.append((off, x.dtype, tuple(x.shape)))
            tensors.append(x)
            off += (x.numel() * x.element_size() + _ALIGN - 1) // _ALIGN * _ALIGN
            return _Slot(len(tensors) - 1)
        if isinstance(x, dict):
            return {k: walk(v) for k, v in x.items()}
        if isinstance(x, list):
            return [walk(v) for v in x]
        if isinstance(x, tuple):
            return tuple(walk(v) for v in x)
        return x

    template = walk(batch)
    pin = torch.cuda.is_available() if pin is None else pin
    buf = torch.empty(max(off, 1), dtype=torch.uint8, pin_memory=pin)
    views = []
    for (o, dtype, shape), t in zip(slots, tensors):
        v = buf[o:o + _nbytes(dtype, shape)].view(dtype).view(shape)
        v.copy_(t)
        views.append(v)
    return PackedBatch(_fill(template, views), buf, template, slots)


def pin_tree(x):
    """Pinned copy of a batch: a dict becomes a :class:`PackedBatch` (one buffer); other trees are pinned
    tensor by tensor."""
    if isinstance(x, PackedBatch):
        return x
    if isinstance(x, dict) and torch.cuda.is_available():
        return pack_tree(x)
    return _pin_each(x)


def _pin_each(x):
    if torch.is_tensor(x):
        return x.pin_memory() if not x.is_pinned() else x
    if isinstance(x, dict):
        return {k: _pin_each(v) for k, v in x.items()}
    if isinstance(x, list):
        return [_pin_each(v) for v in x]
    if isinstance(x, tuple):
        return tuple(_pin_each(v) for v in x)
    return x


def entity_total_hint(batch) -> Optional[int]:
    """Host-side packed entity count of an RL learner batch (sum of min(entity_num, N)), computed from the
    host copy before the H2D transfer; the model uses it to pack entities without a device->host sync."""
    if not isinstance(batch, dict) or not torch.is_tensor(batch.get('entity_num')) or \
            not isinstance(batch.get('entity_info'), dict) or batch['entity_num'].is_cuda:
        return None
    ut = batch['entity_info'].get('unit_type')
    if not torch.is_tensor(ut) or ut.dim() < 2:
        return None
    return int(batch['entity_num'].clamp(max=ut.shape[-1]).sum())


def _to(x, device, stream):
    if torch.is_tensor(x):
        y = x.to(device, non_blocking=True)
        y.record_stream(torch.cuda.current_stream(device))
        return y
    if isinstance(x, dict):
        return {k: _to(v, device, stream) for k, v in x.items()}
    if isinstance(x, list):
        return [_to(v, device, stream) for v in x]
    if isinstance(x, tuple):
        return tuple(_to(v, device, stream) for v in x)
    return x


class DevicePrefetcher:
    """Wrap an iterator of host batches; yields device batches one step ahead."""

    def __init__(self, source: Iterator[Any], device: torch.device):
        self.source = source
        self.device = torch.device(device)
        self.gpu = self.device.type == 'cuda'
        self.stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        self._next: Optional[Any] = None
        self._event = None
        self._stage()

    def _stage(self):
        try:
            host = next(self.source)
        except StopIteration:
            self._next = None
            return
        if not self.gpu:
            self._next = host
            return
        compute = torch.cuda.current_stream(self.device)
        hint = entity_total_hint(host)
        with torch.cuda.stream(self.stream):
            # copies are issued on the side stream; record_stream ties lifetime to the compute stream
            if isinstance(host, PackedBatch) and PACKED_H2D:
                self._next = host.to_device(self.device, record_stream=compute)
            else:
                self._next = _to_side(host, self.device, compute)
            self._event = torch.cuda.Event()
            self._event.record(self.stream)
        if hint is not None:
            self._next['entity_total'] = hint

    def __iter__(self):
        return self

    def __next__(self):
        if self._next is None:
            raise StopIteration
        if self.gpu:
            torch.cuda.current_stream(self.device).wait_event(self._event)
        out = self._next
        self._stage()
        return out


def _to_side(x, device, compute_stream):
    if torch.is_tensor(x):
        y = x.to(device, non_blocking=True)
        y.record_stream(compute_stream)
        return y
    if isinstance(x, dict):
        return {k: _to_side(v, device, compute_stream) for k, v in x.items()}
    if isinstance(x, list):
        return [_to_side(v, device, compute_stream) for v in x]
    if isinstance(x, tuple):
        return tuple(_to_side(v, device, compute_stream) for v in x)
    return x
