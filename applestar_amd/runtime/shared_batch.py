"""Shared-memory batch slabs between a collator process and the learner (the SL data path).

Reference: ``distar/agent/default/sl_training/sl_dataloader.py:19-94`` keeps one shared-memory batch whose rows
the decode workers fill in place, then the main process moves it to the GPU.  Here, MI355X-first:

* ``n_slabs`` fixed-capacity byte slabs in POSIX shared memory (torch shared storage), registered with the
  HIP runtime (``hipHostRegister``) in the learner process, so a slab is DMA-able pinned memory;
* a collator *process* (off the learner's Python thread and GIL) assembles each batch - slot bookkeeping,
  padding, stacking - and packs every tensor of it into a free slab at 64-byte aligned offsets, then
  sends only the small layout (slot table) over a queue;
* the learner rebuilds the batch as views of the slab and issues ONE ``non_blocking`` copy of the used bytes
  on a side HIP stream, one batch ahead of compute; the slab returns to the collator when that copy's event
  has completed (never while the DMA may still read it).

With ``n_slabs = 3`` the collator packs batch i+2 while batch i+1 is in flight and batch i trains.
"""
from __future__ import annotations

import collections
import queue
from typing import Any, Callable, Iterator, Optional

import torch

from .prefetch import PackedBatch, _fill, _nbytes, _Slot, entity_total_hint

_ALIGN = 64


def layout(batch) -> tuple:
    """(template, slots, nbytes) of ``batch`` packed at 64-byte aligned offsets (prefetch.pack_tree order)."""
    slots, tensors = [], []
    off = 0

    def walk(x):
        nonlocal off
        if torch.is_tensor(x):
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
    return template, slots, off, tensors


def pack_into(slab: torch.Tensor, batch) -> tuple:
    """Write every tensor of ``batch`` into the uint8 ``slab``; returns (template, slots, nbytes)."""
    template, slots, nbytes, tensors = layout(batch)
    if nbytes > slab.numel():
        raise RuntimeError(f'shared batch slab too small: batch needs {nbytes >> 20} MiB, slab holds '
                           f'{slab.numel() >> 20} MiB (raise learner.data.slab_mb)')
    for (o, dtype, shape), t in zip(slots, tensors):
        slab[o:o + _nbytes(dtype, shape)].view(dtype).view(shape).copy_(t)
    return template, slots, nbytes


def unpack(slab: torch.Tensor, template, slots, nbytes) -> PackedBatch:
    """The batch as views of ``slab`` (a PackedBatch whose buffer is the used prefix of the slab)."""
    buf = slab[:max(nbytes, 1)]
    views = [buf[o:o + _nbytes(dtype, shape)].view(dtype).view(shape) for o, dtype, shape in slots]
    return PackedBatch(_fill(template, views), buf, template, slots)


def _collator_main(make_batches: Callable[[], Iterator[Any]], slabs, free_q, ready_q):
    torch.set_num_threads(1)
    try:
        for batch in make_batches():
            k = free_q.get()
            if k is None:
                return
            template, slots, nbytes = pack_into(slabs[k], batch)
            ready_q.put((k, template, slots, nbytes))
        ready_q.put(None)
    except Exception as e:          # noqa: BLE001 - surfaced in the learner process
        ready_q.put(('error', repr(e)))


def check_shm_capacity(nbytes: int, path: str = '/dev/shm', margin: int = 64 << 20) -> None:
    """Fail early, with the fix in the message, when the shared-memory filesystem cannot hold the slabs (torch's
    ``share_memory_`` would otherwise die later with a bus error on first touch of an unbacked page)."""
    import os
    import shutil
    if not os.path.isdir(path):
        return
    free = shutil.disk_usage(path).free
    if free < nbytes + margin:
        raise RuntimeError(f'shared batch slabs need {nbytes >> 20} MiB of {path} but only {free >> 20} MiB are '
                           f'free: lower learner.data.slab_mb / n_slabs or enlarge {path}')


class SharedBatchLoader:
    """Iterator of learner batches produced by a collator process through shared, pinned slabs.

    ``make_batches``: a picklable zero-argument callable run INSIDE the collator process that returns an
    iterator of host batches (dicts of CPU tensors).  On CUDA devices batches come back as device tensors
    (one packed H2D copy each, side stream, one ahead); on CPU as private copies of the slab views."""

    def __init__(self, make_batches: Callable[[], Iterator[Any]], device='cpu', n_slabs: int = 3,
                 slab_bytes: int = 256 << 20):
        import torch.multiprocessing as tmp
        self.device = torch.device(device)
        self.gpu = self.device.type == 'cuda'
        check_shm_capacity(int(n_slabs) * int(slab_bytes))
        ctx = tmp.get_context('spawn')
        self.slabs = [torch.empty(int(slab_bytes), dtype=torch.uint8).share_memory_() for _ in range(n_slabs)]
        self._registered = []
        if self.gpu:
            cudart = torch.cuda.cudart()
            for s in self.slabs:     # pin the shared pages for DMA (hipHostRegister)
                if int(cudart.cudaHostRegister(s.data_ptr(), s.numel(), 0)) == 0:
                    self._registered.append(s)
        self._free, self._ready = ctx.Queue(), ctx.Queue()
        for k in range(n_slabs):
            self._free.put(k)
        self._proc = ctx.Process(target=_collator_main, args=(make_batches, self.slabs, self._free, self._ready),
                                 daemon=True, name='applestar-collator')
        self._proc.start()
        self.stream = torch.cuda.Stream(device=self.device) if self.gpu else None
        self._inflight = collections.deque()     # (event, slab) whose H2D copy was issued
        self._next = None
        self._done = False
        if self.gpu:
            self._next = self._stage()

    def _get(self):
        # wait in short slices and keep returning slabs whose H2D copy has finished: with every slab in flight the
        # collator can only produce once one comes back, so a wait that never releases would deadlock.  After
        # ~50 ms with nothing ready, block on the oldest in-flight copy (it was enqueued, so it completes).
        waited = 0.0
        while True:
            self._release_done()
            try:
                item = self._ready.get(timeout=0.05)
                break
            except queue.Empty:
                waited += 0.05
                if self._inflight:
                    self._release_done(block=True)
                if waited >= 5.0:
                    waited = 0.0
                    if not self._proc.is_alive():
                        raise RuntimeError('shared-batch collator process died')
        if item is None:
            return None
        if item[0] == 'error':
            raise RuntimeError(f'shared-batch collator failed: {item[1]}')
        return item

    def _release_done(self, block=False):
        """Return finished slabs to the collator (``block``: also wait for the OLDEST in-flight copy)."""
        while self._inflight and (block or self._inflight[0][0].query()):
            ev, k = self._inflight.popleft()
            ev.synchronize()
            self._free.put(k)
            block = False

    def _stage(self):
        item = self._get()
        if item is None:
            return None
        k, template, slots, nbytes = item
        host = unpack(self.slabs[k], template, slots, nbytes)
        hint = entity_total_hint(host)
        compute = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.stream):
            dev = host.to_device(self.device, record_stream=compute)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._inflight.append((ev, k))
        if hint is not None:
            dev['entity_total'] = hint
        return dev, ev

    def __iter__(self):
        return self

    def __next__(self):
        if self._done:
            raise StopIteration
        if not self.gpu:
            item = self._get()
            if item is None:
                self._done = True
                raise StopIteration
            k, template, slots, nbytes = item
            view = unpack(self.slabs[k], template, slots, nbytes)
            out = _fill(template, [t.clone() for t in _leaves(view, slots, self.slabs[k])])
            self._free.put(k)
            return out
        if self._next is None:
            self._done = True
            raise StopIteration
        out, ev = self._next
        torch.cuda.current_stream(self.device).wait_event(ev)
        self._release_done()
        self._next = self._stage()
        return out

    def close(self):
        try:
            self._free.put(None)
        except Exception:           # noqa: BLE001 - best-effort shutdown
            pass
        if self._proc.is_alive():
            self._proc.terminate()
        self._proc.join(timeout=5)
        if self.gpu:
            self._release_done(block=True)
            torch.cuda.synchronize(self.device)
            cudart = torch.cuda.cudart()
            for s in self._registered:
                cudart.cudaHostUnregister(s.data_ptr())
            self._registered = []


def _leaves(view: PackedBatch, slots, slab):
    return [slab[o:o + _nbytes(dtype, shape)].view(dtype).view(shape) for o, dtype, shape in slots]
