"""Host -> HBM batch staging on a side HIP stream.

The learner's next batch is copied from pinned host memory with ``non_blocking`` copies issued on a
dedicated copy stream while the current step computes (the reference does this in a separate
process with its own CUDA stream and a multiprocessing queue, ``rl_dataloader.py:113-127,160-169``).
The compute stream waits on an event recorded after the copies, and every staged tensor is marked
``record_stream`` so the caching allocator does not recycle it early.
"""
from __future__ import annotations

from typing import Any, Iterator, Optional

import torch


def pin_tree(x):
    if torch.is_tensor(x):
        return x.pin_memory() if not x.is_pinned() else x
    if isinstance(x, dict):
        return {k: pin_tree(v) for k, v in x.items()}
    if isinstance(x, list):
        return [pin_tree(v) for v in x]
    if isinstance(x, tuple):
        return tuple(pin_tree(v) for v in x)
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
