"""Learner data pipelines.

``RLDataLoader`` (``rl_dataloader.py:79-245``): background threads pull trajectories for
``<player>traj`` from the data plane into a replay buffer of ``buffer_size`` trajectories; each batch
takes ``batch_size`` of them; the remainder is shuffled and topped up with new data that is inserted
twice (``new + old + new``), so each trajectory is reused ~2x exactly like the reference.  Collation
(:func:`collate_trajectories`) happens on the pulling thread, the batch is pinned, and the H2D copy
runs on a side HIP stream one batch ahead of compute (:class:`DevicePrefetcher`).

``SyntheticRLDataLoader`` / ``FakeSLDataLoader``: synthetic batches with the exact learner layout
(``sl_dataloader.py:167-189`` FakeDataloader) for benchmarks and tests.
"""
from __future__ import annotations

import logging
import os
import queue
import random
import threading
from typing import Iterator, List, Optional

import torch

from ..agent.collate import collate_trajectories
from ..runtime.prefetch import DevicePrefetcher, pin_tree


class RLDataLoader:
    """Replay buffer over the data plane.  On a GPU the trajectories live in an HBM
    :class:`TrajectoryRing` and batches are assembled on device; on CPU (tests) the host collate path
    is used.  Both keep the reference's reuse policy (each trajectory trains ~``max_reuse`` times)."""

    def __init__(self, adapter, player_id: str, batch_size: int, buffer_size: Optional[int] = None,
                 device='cpu', queue_size: int = 2, pull_timeout: Optional[float] = None, seed: int = 0,
                 ring_bytes: Optional[int] = None, max_reuse: int = 2, device_collate: Optional[bool] = None):
        self._adapter = adapter
        self._token = player_id + 'traj'
        self.batch_size = int(batch_size)
        self.buffer_size = max(int(buffer_size or batch_size), self.batch_size)
        self.max_reuse = int(max_reuse)
        self._q: queue.Queue = queue.Queue(maxsize=queue_size)
        self._stop = threading.Event()
        self._rng = random.Random(seed)
        self._timeout = pull_timeout
        self.device = torch.device(device)
        self.device_collate = (self.device.type == 'cuda') if device_collate is None else device_collate
        if self.device_collate:
            from ..runtime.traj_ring import TrajectoryRing, auto_ring_bytes
            self._ring = TrajectoryRing(ring_bytes or auto_ring_bytes(self.device), self.device)
            self._avail = threading.Condition()
            self._thread = threading.Thread(target=self._ring_loop, daemon=True, name='rl-ring-ingest')
            self._thread.start()
            self._iter = self._ring_batches()
        else:
            self._thread = threading.Thread(target=self._loop, daemon=True, name='rl-dataloader')
            self._thread.start()
            self._iter = DevicePrefetcher(self._host_batches(), self.device) if self.device.type == 'cuda' else \
                self._host_batches()

    def _pull(self, n: int, raw: bool = False, alloc=None) -> List:
        out: List = []
        while len(out) < n and not self._stop.is_set():
            try:
                out += self._adapter.pull(self._token, size=n - len(out), block=True, sleep_time=0.1, timeout=1.0,
                                          raw=raw, alloc=alloc)
            except (ConnectionError, OSError):  # coordinator restarting / shutting down: retry until stopped
                self._stop.wait(1.0)
        return out

    # ---------------------------------------------------------------- HBM ring path
    def _ring_loop(self):
        torch.set_num_threads(1)
        # diagnostics (tools/bench_pipeline.py): 'discard' keeps receiving once the ring is full but drops the frames
        # (receive cost without the ring insert / H2D copy); 'unpinned' receives into pageable memory
        mode = os.environ.get('APPLESTAR_RING_DIAG', '')
        ring = self._ring        # this thread's ring: close() drops self._ring only once the thread has exited
        while not self._stop.is_set():
            if mode == 'discard' and len(ring) >= self.buffer_size:
                self._pull(1, raw=True)
                continue
            with self._avail:
                while len(ring) >= self.buffer_size and not self._stop.is_set():
                    self._avail.wait(0.5)
            alloc = None if mode == 'unpinned' else ring.stage      # bytes land in pinned staging
            for frame in self._pull(1, raw=True, alloc=alloc):
                if self._stop.is_set():
                    break
                ring.put(frame)
                with self._avail:
                    self._avail.notify_all()

    def _ring_batches(self) -> Iterator:
        while True:
            with self._avail:
                while len(self._ring) < self.batch_size:
                    self._avail.wait(0.5)
            ids = self._ring.least_used(self.batch_size)
            batch = self._ring.batch(ids)
            for tid in ids:
                if self._ring._trajs.get(tid) is not None and self._ring._trajs[tid].uses >= self.max_reuse:
                    self._ring.drop(tid)
            with self._avail:
                self._avail.notify_all()
            yield batch

    # ---------------------------------------------------------------- host path
    def _loop(self):
        torch.set_num_threads(1)
        data = self._pull(self.buffer_size)
        data = data + data[:self.batch_size // 2 + 1]
        while not self._stop.is_set():
            batch = collate_trajectories(data[:self.batch_size])
            if self.device.type == 'cuda':
                batch = pin_tree(batch)
            while not self._stop.is_set():
                try:
                    self._q.put(batch, timeout=0.5)
                    break
                except queue.Full:
                    continue
            data = data[self.batch_size:]
            self._rng.shuffle(data)
            left = self.buffer_size - len(data)
            if left > 0:
                new = self._pull(left)
                data = new + data + new

    def _host_batches(self) -> Iterator:
        while True:
            yield self._q.get()

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._iter)

    @property
    def ring_bytes(self) -> Optional[int]:
        """The HBM ring's capacity (None on the host path or after close): a rebuilt loader reuses it."""
        ring = getattr(self, '_ring', None)
        return ring.capacity if ring is not None else None

    def close(self, timeout: float = 5.0) -> bool:
        """Stop the ingest thread, wait for it, and release the HBM ring (its arena goes back to the caching
        allocator; the caller may ``torch.cuda.empty_cache()`` before sizing a new ring from free memory).
        Returns False when the thread did not exit within ``timeout``: the ring is then kept (the thread may still
        be inserting a frame into it) and freed by a later ``close``."""
        self._stop.set()
        if getattr(self, '_avail', None) is not None:
            with self._avail:
                self._avail.notify_all()
        t = getattr(self, '_thread', None)
        if t is not None and t.is_alive() and t is not threading.current_thread():
            t.join(timeout)
            if t.is_alive():
                logging.getLogger(__name__).warning(
                    'RLDataLoader.close: ingest thread still running after %.1f s; keeping its ring', timeout)
                self._iter = iter(())
                return False
        self._iter = iter(())
        if getattr(self, '_ring', None) is not None:
            self._ring = None
        return True


class SyntheticRLDataLoader:
    """Endless synthetic RL batches (fixed seed set, cycled) moved to ``device``."""

    def __init__(self, batch_size: int, unroll_len: int, device='cpu', use_value_feature: bool = True,
                 n_distinct: int = 2, max_entities: int = 512):
        from ..rl.synthetic import rl_batch
        self._batches = [pin_tree(rl_batch(batch_size, unroll_len, max_entities=max_entities, seed=s,
                                           use_value_feature=use_value_feature))
                         if torch.device(device).type == 'cuda' else
                         rl_batch(batch_size, unroll_len, max_entities=max_entities, seed=s,
                                  use_value_feature=use_value_feature) for s in range(n_distinct)]
        self.device = torch.device(device)

        def gen():
            i = 0
            while True:
                yield self._batches[i % len(self._batches)]
                i += 1
        self._iter = DevicePrefetcher(gen(), self.device) if self.device.type == 'cuda' else gen()

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._iter)


class FakeSLDataLoader:
    """Synthetic supervised batches (``FakeDataloader``), batch-major [B*T]."""

    def __init__(self, batch_size: int, traj_len: int, device='cpu', n_distinct: int = 2, max_entities: int = 512):
        from ..rl.synthetic import sl_batch, to_device
        self._batches = [sl_batch(batch_size, traj_len, max_entities=max_entities, seed=s)
                         for s in range(n_distinct)]
        self.device = torch.device(device)
        self._to = to_device
        self._i = 0

    def __iter__(self):
        return self

    def __next__(self):
        b = self._batches[self._i % len(self._batches)]
        self._i += 1
        return self._to(b, self.device) if self.device.type != 'cpu' else b
