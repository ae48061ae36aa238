"""HBM-resident trajectory ring with on-device batch assembly.

The reference learner unpickles every trajectory on the host, pads and stacks it with per-tensor
Python collate and copies the batch to the GPU (``rl_dataloader.py:45-127``) — ~2 s of host work
per 6x64 batch here, ~25x a learner step.  Instead:

* ``put(frame)``: a trajectory arrives as one :mod:`utils.serialize` frame (list of T+1 step
  dicts).  Its JSON header is parsed (no tensor decoding) into per-leaf descriptors and the raw
  body is copied ONCE, host pinned staging -> HBM arena, on a dedicated copy stream.  The arena
  is a ring (oldest trajectories are evicted when it wraps); 288 GB/GPU holds ~10^4 trajectories.
* ``batch(ids)``: the padded learner batch (``collate_trajectories`` layout: observations
  time-major (T+1)*B padded to the batch max entity count, actions/logits [T,B,...], SU / target
  logits padded with -1e9, masks) is assembled by ONE ``segment_copy`` kernel launch that moves
  every row of every leaf of every step from the arena into one pre-filled batch buffer; masks are
  derived on device.  Host work is numpy arithmetic on descriptor tables.
* reuse: trajectories stay resident, so the reference's ~2x replay reuse costs no copies.
"""
from __future__ import annotations

import threading
import warnings
from collections import OrderedDict, deque
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..lib.features import MAX_SELECTED_UNITS_NUM
from ..utils import serialize

NEG = -1e9
_ALIGN = 256
OBS_TOP = ('spatial_info', 'entity_info', 'scalar_info', 'entity_num', 'value_feature')
NEG_FILL = {('behaviour_logp', 'selected_units'), ('teacher_logit', 'selected_units'), ('teacher_logit', 'target_unit'),
            ('successive_logit', 'selected_units'), ('successive_logit', 'target_unit')}
SU_PAD = {('action_info', 'selected_units'), ('behaviour_logp', 'selected_units')}
SU_2D = {('teacher_logit', 'selected_units'), ('successive_logit', 'selected_units')}
ENTITY_N = {('teacher_logit', 'target_unit'), ('successive_logit', 'target_unit')}


def _leaves(node, path=()):
    """Yield (path, descriptor) for every tensor leaf of a header tree (hidden_state indexed by ints)."""
    if '__t__' in node:
        yield path, node['__t__']
    elif '__d__' in node:
        for k, v in node['__d__']:
            yield from _leaves(v, path + (k,))
    elif '__l__' in node or '__tu__' in node:
        for i, v in enumerate(node.get('__l__', node.get('__tu__'))):
            yield from _leaves(v, path + (i,))


_W = 7   # per-leaf index row: body offset, nbytes, ndim, 4 dims (csrc/codec.cpp traj_index)


class _Traj:
    """A resident trajectory: its arena extent and its leaf index - ``paths`` (leaf paths of a step), ``dts`` (dtype
    codes), ``meta`` int64 [T + 1, leaves, 7] (offset into the frame body, nbytes, ndim, dims)."""
    __slots__ = ('start', 'size', 'T', 'paths', 'pidx', 'dts', 'meta', 'entity_counts', 'event', 'uses')

    def __init__(self, start, size, paths, dts, meta):
        self.start, self.size = start, size
        self.T = meta.shape[0] - 1
        self.paths, self.dts, self.meta = paths, dts, meta
        self.pidx = {p: i for i, p in enumerate(paths)}
        ex = self.pidx[('entity_info', 'x')]
        self.entity_counts = meta[:, ex, 3].copy()
        self.event = None
        self.uses = 0


def _index_py(steps):
    """Python form of csrc/codec.cpp traj_index over a parsed header's step list (fallback): the union of the steps'
    leaves in first-seen order, nbytes -1 where a step lacks a leaf."""
    pos, paths, dts, rows = {}, [], [], []
    for t, st in enumerate(steps):
        for path, d in _leaves(st):
            if path not in pos:
                pos[path] = len(paths)
                paths.append(path)
                dts.append(d[0])
            elif dts[pos[path]] != d[0]:
                raise ValueError(f'trajectory leaf {path} changes dtype')
            rows.append((t, pos[path], d))
    meta = np.ones((len(steps), len(paths), _W), dtype=np.int64)
    meta[:, :, 0], meta[:, :, 1], meta[:, :, 2] = 0, -1, 0
    for t, i, d in rows:
        shape = list(d[1])
        if len(shape) > _W - 3:
            raise ValueError('trajectory leaf with more than 4 dims')
        meta[t, i, 0], meta[t, i, 1], meta[t, i, 2] = d[2], d[3], len(shape)
        meta[t, i, 3:3 + len(shape)] = shape
    return paths, dts, meta


def _native_index(frame):
    """csrc/codec.cpp traj_index (the header parsed with the GIL released), or None (extension missing, compressed
    frame, a leaf the table cannot hold) - the caller parses in Python."""
    try:
        from ..ops import native
        C = native._C if native._C is not None else native.ensure_loaded()
    except Exception:   # noqa: BLE001 - CPU-only installs without the extension
        return None
    fn = getattr(C, 'traj_index', None)
    if fn is None or len(frame) <= len(serialize.MAGIC) + 8 or memoryview(frame)[len(serialize.MAGIC) + 8] != 0:
        return None
    r = fn(frame)
    if r is None:
        return None
    paths, dts, meta, body_off = r
    return [tuple(p) for p in paths], list(dts), meta, int(body_off)


def auto_ring_bytes(device, step_peak_gb: float = 20.0, headroom_gb: float = 8.0, fraction: float = 0.75,
                    min_gb: float = 1.0, max_gb: Optional[float] = None) -> int:
    """HBM ring size from what the device has free: ``fraction`` x (free - learner step peak - headroom).

    The fp32 learner step peaks at 15.1 GB of HBM (B = 6, T = 64; bench.py's ``peak_mem_gb``), the bf16 step
    lower, so the default ``step_peak_gb`` of 20 GB leaves a margin; on an MI355X (288 GB) with the learner
    alone that is ~195 GB of trajectories - ~6,000 T = 64 trajectories of ~30 MB at 512 entities - instead of a
    fixed 16 GB.  ``fraction`` < 1 leaves room for an inference server sharing the GPU.  Call before the model's
    first step (the free memory then does not include the step's activations yet)."""
    dev = torch.device(device)
    if dev.type != 'cuda':
        return int(min_gb * (1 << 30))
    free, _ = torch.cuda.mem_get_info(dev)
    avail = free - (step_peak_gb + headroom_gb) * (1 << 30)
    n = max(avail * fraction, min_gb * (1 << 30))
    if max_gb is not None:
        n = min(n, max_gb * (1 << 30))
    return int(n) // (1 << 20) * (1 << 20)


class TrajectoryRing:
    def __init__(self, capacity_bytes: int, device='cuda', staging_buffers: int = 4):
        self.device = torch.device(device)
        self.capacity = int(capacity_bytes)
        self.arena = torch.empty(self.capacity, dtype=torch.uint8, device=self.device)
        self._head = 0
        self._trajs: 'OrderedDict[int, _Traj]' = OrderedDict()
        self._next_id = 0
        self._lock = threading.Lock()
        cuda = self.device.type == 'cuda'
        self._stream = torch.cuda.Stream(self.device) if cuda else None
        self._staging = deque([[None, None] for _ in range(staging_buffers)])  # [pinned tensor, event]
        self._native = None
        if cuda:
            from ..ops import native
            native.ensure_loaded()
            self._native = native._C

    # ------------------------------------------------------------------ ingest
    def _alloc(self, size: int) -> int:
        size = (size + _ALIGN - 1) // _ALIGN * _ALIGN
        if size > self.capacity:
            raise ValueError(f'trajectory of {size} B exceeds the ring ({self.capacity} B)')
        start = self._head if self._head + size <= self.capacity else 0
        end = start + size
        for tid in [k for k, tr in self._trajs.items() if tr.start < end and start < tr.start + tr.size]:
            del self._trajs[tid]  # overwritten: evict
        self._head = end
        return start

    def _next_slot(self, n: int):
        slot = self._staging[0]
        self._staging.rotate(-1)
        if slot[1] is not None:
            slot[1].synchronize()  # the previous async copy out of this staging buffer has finished
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(max(n, 1 << 20), dtype=torch.uint8, pin_memory=self._stream is not None)
        return slot

    def stage(self, n: int):
        """Receive target for a frame of ``n`` bytes (pass as ``alloc`` to ``Adapter.pull``): a pinned
        staging buffer, so :meth:`put` can DMA it to HBM without another host copy."""
        slot = self._next_slot(n)
        view = memoryview(slot[0].numpy())[:n]
        self._staged = (view, slot)
        return view

    def put(self, frame) -> int:
        staged = getattr(self, '_staged', None)
        slot = staged[1] if staged is not None and frame is staged[0] else None
        self._staged = None
        idx = _native_index(frame)
        if idx is not None:
            paths, dts, meta, body_off = idx
            body = memoryview(frame)[body_off:]
        else:
            header, body = serialize.parse(frame)
            paths, dts, meta = _index_py(header['__l__'])
        n = len(body)
        body_off = len(frame) - n
        with self._lock:
            start = self._alloc(n)
            tr = _Traj(start, (n + _ALIGN - 1) // _ALIGN * _ALIGN, paths, dts, meta)
            if slot is None:
                with warnings.catch_warnings():  # read-only source: only ever copied from
                    warnings.simplefilter('ignore')
                    src = torch.frombuffer(body, dtype=torch.uint8) if n else torch.empty(0, dtype=torch.uint8)
            if self._stream is None:
                self.arena[start:start + n].copy_(src if slot is None else slot[0][body_off:body_off + n])
            else:
                if slot is None:
                    slot = self._next_slot(n)
                    slot[0][:n].copy_(src)
                    body_off = 0
                with torch.cuda.stream(self._stream):
                    self.arena[start:start + n].copy_(slot[0][body_off:body_off + n], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._stream)
                slot[1] = ev
                tr.event = ev
            tid = self._next_id
            self._next_id += 1
            self._trajs[tid] = tr
            return tid

    def __len__(self):
        return len(self._trajs)

    def ids(self) -> List[int]:
        return list(self._trajs)

    def least_used(self, k: int) -> List[int]:
        with self._lock:
            order = sorted(self._trajs.items(), key=lambda kv: (kv[1].uses, kv[0]))
            return [tid for tid, _ in order[:k]]

    def drop(self, tid: int) -> None:
        with self._lock:
            self._trajs.pop(tid, None)

    # ------------------------------------------------------------------ batch assembly
    def batch(self, ids: Sequence[int]) -> Dict:
        with self._lock:
            trs = [self._trajs[i] for i in ids]
            for tr in trs:
                tr.uses += 1
        B, T = len(trs), trs[0].T
        assert all(tr.T == T for tr in trs), 'trajectories in a batch must share the unroll length'
        N = int(max(tr.entity_counts.max() for tr in trs))
        layout, segs = [], []
        offset = 0
        t0 = trs[0]
        for li0, path in enumerate(t0.paths):
            if t0.meta[0, li0, 1] < 0:       # absent in the first step of the first trajectory
                continue
            dt = serialize.DTYPES[t0.dts[li0]]
            esize = torch.empty(0, dtype=torch.uint8 if dt == torch.bool else dt).element_size()
            is_obs = path[0] in OBS_TOP
            is_hidden = path[0] == 'hidden_state'
            steps = 1 if is_hidden else (T + 1 if is_obs else T)
            if path[0] == 'entity_info':
                row_shape = (N,)
            elif path in SU_PAD:
                row_shape = (MAX_SELECTED_UNITS_NUM,)
            elif path in SU_2D:
                row_shape = (MAX_SELECTED_UNITS_NUM, N + 1)
            elif path in ENTITY_N:
                row_shape = (N,)
            else:
                m0 = t0.meta[0, li0]
                row_shape = tuple(int(x) for x in m0[3:3 + m0[2]])
            row_bytes = int(np.prod(row_shape, dtype=np.int64)) * esize
            offset = (offset + _ALIGN - 1) // _ALIGN * _ALIGN
            layout.append((path, dt, (steps * B,) + row_shape, offset, steps))
            rows = np.arange(steps, dtype=np.int64) * B
            # per (t, b) segments
            for b, tr in enumerate(trs):
                m = tr.meta[:steps, tr.pidx[path]]            # [steps, 7]
                offs = m[:, 0] + tr.start
                nb = m[:, 1]
                dst = offset + (rows + b) * row_bytes
                if path in SU_2D:  # [s, n+1] -> [64, N+1]: one segment per source row
                    two = (m[:, 2] == 2) & (nb > 0)
                    for t in np.nonzero(two)[0]:
                        s_, c = int(m[t, 3]), int(m[t, 4])
                        if s_ == 0:
                            continue
                        r = np.arange(s_, dtype=np.int64)
                        segs.append(np.stack([offs[t] + r * c * esize, dst[t] + r * (N + 1) * esize,
                                              np.full(s_, c * esize, dtype=np.int64)], 1))
                else:
                    keep = nb > 0
                    segs.append(np.stack([offs[keep], dst[keep], nb[keep]], 1))
            offset += steps * B * row_bytes
        total = max(offset, 1)
        seg = np.concatenate(segs, 0) if segs else np.zeros((0, 3), dtype=np.int64)
        # bounds check on the host before any device access (kernel reads arena[src:src+n])
        if len(seg):
            assert seg[:, 0].min() >= 0 and (seg[:, 0] + seg[:, 2]).max() <= self.capacity
            assert seg[:, 1].min() >= 0 and (seg[:, 1] + seg[:, 2]).max() <= total
        buf = torch.zeros(total, dtype=torch.uint8, device=self.device)
        out = {}
        for path, dt, shape, off, steps in layout:
            store = torch.uint8 if dt == torch.bool else dt
            n = int(np.prod(shape, dtype=np.int64))
            es = torch.empty(0, dtype=store).element_size()
            view = buf[off:off + n * es].view(store).view(shape)
            if path in NEG_FILL:
                view.fill_(NEG)
            out[path] = view.view(torch.bool) if dt == torch.bool else view
        if self._stream is not None:
            cur = torch.cuda.current_stream(self.device)
            for tr in trs:
                if tr.event is not None:
                    cur.wait_event(tr.event)
        if len(seg):
            seg_t = torch.from_numpy(seg)
            if self.device.type == 'cuda':
                seg_t = seg_t.pin_memory().to(self.device, non_blocking=True)
                self._native.segment_copy(self.arena, buf, seg_t)
            else:  # host fallback (tests): same semantics
                a = self.arena.numpy()
                o = buf.numpy()
                for s_, d_, n_ in seg:
                    o[d_:d_ + n_] = a[s_:s_ + n_]
        return self._tree(out, B, T, N)

    @staticmethod
    def _tree(flat: Dict[tuple, torch.Tensor], B: int, T: int, N: int) -> Dict:
        batch: Dict = {}
        hidden: Dict[int, Dict[int, torch.Tensor]] = {}
        for path, t in flat.items():
            if path[0] == 'hidden_state':
                hidden.setdefault(path[1], {})[path[2]] = t
                continue
            if path[0] not in OBS_TOP:
                t = t.view(T, B, *t.shape[1:])
            node = batch
            for k in path[:-1]:
                node = node.setdefault(k, {})
            node[path[-1]] = t
        if hidden:
            batch['hidden_state'] = [(hidden[l][0], hidden[l][1]) for l in sorted(hidden)]
        en = batch['entity_num'].view(T + 1, B)[:T].long()
        dev = en.device
        m = batch.setdefault('mask', {})
        if 'selected_units_num' in batch:
            m['selected_units_mask'] = torch.arange(MAX_SELECTED_UNITS_NUM, device=dev) < \
                batch['selected_units_num'].long().unsqueeze(-1)
        m['selected_units_logits_mask'] = torch.arange(N + 1, device=dev) < (en + 1).unsqueeze(-1)
        m['target_units_logits_mask'] = torch.arange(N, device=dev) < en.unsqueeze(-1)
        batch['batch_size'] = B
        batch['unroll_len'] = T
        return batch
