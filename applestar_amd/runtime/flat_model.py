"""Learner -> actor model hand-off as ONE flat buffer with a version counter ("Learner -> actor models:
shared host buffer plus a version counter; a device-to-device copy serves the co-located inference server").

The reference copies the policy state_dict into a shared-memory ``model_ref``, then ``torch.save`` + lz4 + TCP
every 4 iterations (``distar/ctools/worker/learner/learner_comm.py:53-99``); actors pull and ``load_state_dict``
(``actor_comm.py:172-216``).  Here:

* :class:`FlatLayout` - the policy tensors' fixed order / shapes / offsets in one fp32 vector (every policy tensor
  is fp32: parameters and the frozen tables alike);
* :class:`ModelPublisher` (learner) - ``publish``: ONE native multi-tensor copy (device, stream-ordered behind the
  optimizer step) of every policy tensor into a flat device buffer, then ONE D2H DMA into a pinned host buffer on
  a side stream.  The host buffer is either private (the cross-host path pushes it as a single tensor over the
  data plane) or a :class:`SharedModelSlot` in ``/dev/shm`` that co-located inference servers read directly;
* :class:`SharedModelSlot` - POSIX shared memory: a 64-byte header (seqlock ``version``: odd while a copy is in
  flight; ``model_last_iter``; ``reset_flag``; payload size; the publisher's random ``session`` id; a hash of the
  layout's names and shapes; the publisher's pid) followed by the flat fp32 payload, registered with the HIP runtime
  (``hipHostRegister``) in every process that maps it, so both the learner's D2H and the reader's H2D are DMAs;
* :class:`ModelSubscriber` (inference server) - ``poll``: when the version moved, ONE H2D DMA of the flat payload
  into a device buffer, a version re-check (a torn read is dropped and retried next poll), then ONE native
  multi-tensor D2D copy into the resident model's parameters (captured HIP graphs stay valid: the parameters are
  updated in place).  A subscriber is bound to ONE publisher session: ``poll`` reports the slot ``stale`` when the
  file was replaced (another inode at the path: a restarted learner, ``reset_comm_setting``), when a new publisher
  re-created it in place (another session id), when the layout hash no longer matches or when the publishing
  process has exited (a slot left behind by a crashed or terminated learner is never attached either: it would
  serve that run's last weights to the next run's actors); the caller then re-attaches or falls back to the network
  broadcast (actor/comm.py).

A ~116 MB policy moves as one DMA each way instead of ~430 per-tensor copies, a clone and a pickle/TCP frame.
"""
from __future__ import annotations

import hashlib
import mmap
import os
import struct
import threading
from typing import Dict, List, Optional, Tuple

import torch

_HEADER = 64
# version, model_last_iter, reset_flag, payload elements, session, layout hash, publisher pid
_HDR = struct.Struct('<qqqqQQq')


class FlatLayout:
    """Fixed (name, shape, offset) order of a state dict's fp32 tensors in one flat vector."""

    def __init__(self, state_dict: Dict[str, torch.Tensor]):
        self.names: List[str] = []
        self.shapes: List[Tuple[int, ...]] = []
        self.offsets: List[int] = []
        off = 0
        for k, v in state_dict.items():
            if v.dtype != torch.float32:
                raise TypeError(f'FlatLayout: {k} is {v.dtype}; the hand-off carries fp32 tensors only')
            self.names.append(k)
            self.shapes.append(tuple(v.shape))
            self.offsets.append(off)
            off += v.numel()
        self.numel = off

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for k, s, o in zip(self.names, self.shapes, self.offsets):
            n = 1
            for d in s:
                n *= d
            out[k] = flat[o:o + n].view(s)
        return out

    def signature(self) -> Tuple:
        return tuple(zip(self.names, self.shapes))

    def digest(self) -> int:
        """64-bit hash of the (name, shape) order: two layouts with equal element counts but different tensors
        never match."""
        h = hashlib.blake2b(digest_size=8)
        for k, s in zip(self.names, self.shapes):
            h.update(k.encode())
            h.update(struct.pack(f'<{len(s) + 1}q', len(s), *s))
        return int.from_bytes(h.digest(), 'little')


def _copy_many(dsts: List[torch.Tensor], srcs: List[torch.Tensor]) -> None:
    """One native multi-tensor launch on GPU tensors (torch foreach copy elsewhere).  Pairs whose strides differ
    (a channels_last conv weight against its contiguous flat view) fall back to a per-tensor copy inside
    ``multi_copy``: same values, logical order."""
    if dsts and dsts[0].is_cuda and srcs[0].is_cuda:
        from ..ops import native
        native.ensure_loaded().multi_copy(dsts, srcs)
    else:
        for d, s in zip(dsts, srcs):
            d.copy_(s)


class SharedModelSlot:
    """``/dev/shm/<name>``: 64-B header + ``numel`` fp32 payload; pinned (hipHostRegister) in this process."""

    def __init__(self, name: str, numel: int, create: bool = False, layout_hash: int = 0):
        self.path = os.path.join('/dev/shm', name)
        nbytes = _HEADER + 4 * int(numel)
        if create:
            from .shared_batch import check_shm_capacity
            check_shm_capacity(nbytes)
            fd = os.open(self.path, os.O_CREAT | os.O_RDWR, 0o600)
            os.ftruncate(fd, nbytes)
        else:
            fd = os.open(self.path, os.O_RDWR)
            if os.fstat(fd).st_size < nbytes:
                os.close(fd)
                raise ValueError(f'{self.path} holds fewer than {numel} elements')
        self._mm = mmap.mmap(fd, nbytes)
        self.inode = os.fstat(fd).st_ino
        os.close(fd)
        self.numel = int(numel)
        self.session = int.from_bytes(os.urandom(8), 'little') if create else 0
        self.layout_hash = int(layout_hash)
        self.owner_pid = os.getpid() if create else 0
        buf = torch.frombuffer(self._mm, dtype=torch.uint8)
        self.header = buf[:_HEADER]
        self.payload = buf[_HEADER:].view(torch.float32)
        if create:
            self._write_header(0, 0, 0)
        else:
            self.session, self.layout_hash, self.owner_pid = self.read_header()[4:7]
        self._registered = False
        if torch.cuda.is_available():
            rc = int(torch.cuda.cudart().cudaHostRegister(buf.data_ptr(), nbytes, 0))
            self._registered = rc == 0
        self._base = buf

    def _write_header(self, version: int, last_iter: int, reset: int) -> None:
        self._mm[0:_HDR.size] = _HDR.pack(int(version), int(last_iter), int(reset), self.numel, self.session,
                                          self.layout_hash, self.owner_pid)

    def read_header(self) -> Tuple[int, int, int, int, int, int, int]:
        return _HDR.unpack(self._mm[0:_HDR.size])

    def owner_alive(self) -> bool:
        """The publishing process still runs (co-located: one pid namespace)."""
        pid = int(self.read_header()[6])
        if pid <= 0:
            return False
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            return False
        except PermissionError:       # exists, another user's
            return True
        return True

    def replaced(self) -> bool:
        """True when the path no longer names the mapped file (unlinked, or re-created as another inode)."""
        try:
            return os.stat(self.path).st_ino != self.inode
        except FileNotFoundError:
            return True

    def begin_write(self) -> int:
        v = self.read_header()[0]
        self._mm[0:8] = struct.pack('<q', v + 1 if v % 2 == 0 else v)     # odd: a copy is in flight
        return v

    def end_write(self, last_iter: int, reset: bool) -> int:
        v = self.read_header()[0]
        v = v + 1 if v % 2 else v + 2
        self._write_header(v, last_iter, 1 if reset else 0)
        return v

    def close(self, unlink: bool = False) -> None:
        if self._registered:
            torch.cuda.cudart().cudaHostUnregister(self._base.data_ptr())
            self._registered = False
        self.header = self.payload = self._base = None
        try:
            self._mm.close()
        except BufferError:      # a view still exported somewhere: leave the mapping to the GC
            pass
        if unlink and os.path.exists(self.path):
            os.unlink(self.path)


class ModelPublisher:
    """Learner side.  ``shm_name``: also publish into a :class:`SharedModelSlot` for co-located readers."""

    def __init__(self, state_dict: Dict[str, torch.Tensor], shm_name: Optional[str] = None):
        self.layout = FlatLayout(state_dict)
        dev = next(iter(state_dict.values())).device
        self.device = dev
        self.flat_dev = torch.empty(self.layout.numel, dtype=torch.float32, device=dev)
        self.slot = SharedModelSlot(shm_name, self.layout.numel, create=True,
                                    layout_hash=self.layout.digest()) if shm_name else None
        if self.slot is not None:
            self.flat_host = self.slot.payload
        else:
            self.flat_host = torch.empty(self.layout.numel, dtype=torch.float32, pin_memory=dev.type == 'cuda')
        self._stream = torch.cuda.Stream(dev) if dev.type == 'cuda' else None
        self._event = None
        self._meta = (0, False)
        self.version = 0
        self._lock = threading.Lock()

    def publish(self, state_dict: Dict[str, torch.Tensor], last_iter: int = 0, reset_flag: bool = False) -> None:
        """Stream-ordered snapshot: one multi-copy into the flat device buffer (on the current stream, after the
        optimizer step) and one D2H DMA on a side stream; ``wait()`` completes it."""
        views = self.layout.views(self.flat_dev)
        dsts, srcs = [], []
        for k in self.layout.names:
            dsts.append(views[k])
            srcs.append(state_dict[k].detach())
        with self._lock:
            if self._event is not None:
                self._event.synchronize()        # the previous D2H still reads flat_host / flat_dev
            _copy_many(dsts, srcs)
            if self.slot is not None:
                self.slot.begin_write()
            if self._stream is not None:
                self._stream.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(self._stream):
                    self.flat_host.copy_(self.flat_dev, non_blocking=True)
                    self._event = torch.cuda.Event()
                    self._event.record(self._stream)
            else:
                self.flat_host.copy_(self.flat_dev)
                self._event = None
            self._meta = (int(last_iter), bool(reset_flag))
            self.version += 1

    def wait(self) -> Tuple[torch.Tensor, int, bool]:
        """Block until the last publish landed in host memory; stamps the shared slot's version.  Returns the host
        buffer (shared with the next publish: clone to keep), model_last_iter and reset_flag."""
        with self._lock:
            if self._event is not None:
                self._event.synchronize()
                self._event = None
            if self.slot is not None and self.slot.read_header()[0] % 2:
                self.slot.end_write(*self._meta)
            return self.flat_host, self._meta[0], self._meta[1]

    def payload(self) -> Dict:
        """The cross-host message: one flat tensor + the layout (a data-plane frame of one tensor)."""
        flat, it, reset = self.wait()
        return {'flat_model': flat.clone(), 'names': list(self.layout.names),
                'shapes': [list(s) for s in self.layout.shapes], 'model_last_iter': it, 'reset_flag': reset}

    def close(self, unlink: bool = True) -> None:
        self.wait()
        if self.slot is not None:
            self.slot.close(unlink=unlink)


class ModelSubscriber:
    """Inference-server side: keeps ``model``'s tensors equal to the newest published version."""

    def __init__(self, model: torch.nn.Module, shm_name: str, device=None):
        self._targets = dict(model.state_dict())
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        self.slot = SharedModelSlot(shm_name, self._numel_of(shm_name), create=False)
        self.layout: Optional[FlatLayout] = None
        self.version = 0
        self.last_iter = 0
        self.reset_flag = False
        self.flat_dev = torch.empty(self.slot.numel, dtype=torch.float32, device=self.device)
        self._dsts: List[torch.Tensor] = []
        self._srcs: List[torch.Tensor] = []
        self.stale = not self.slot.owner_alive()     # a dead learner's slot is never read

    @staticmethod
    def _numel_of(shm_name: str) -> int:
        with open(os.path.join('/dev/shm', shm_name), 'rb') as f:
            return _HDR.unpack(f.read(_HDR.size))[3]

    def bind(self, layout: FlatLayout) -> None:
        """The publisher's layout (e.g. built from the same model class's policy state dict); only tensors
        present in the resident model with equal shapes are updated.  The slot must carry the same layout
        (element count AND the hash of every name and shape)."""
        if layout.numel != self.slot.numel or layout.digest() != self.slot.layout_hash:
            raise ValueError('ModelSubscriber: layout does not match the shared slot')
        self.layout = layout
        views = layout.views(self.flat_dev)
        self._dsts, self._srcs = [], []
        for k, shp in zip(layout.names, layout.shapes):
            t = self._targets.get(k)
            if t is not None and tuple(t.shape) == tuple(shp):
                self._dsts.append(t)
                self._srcs.append(views[k])

    def poll(self) -> bool:
        """Load the newest version if one was published since the last poll; True when the model changed."""
        if self.layout is None or self.stale:
            return False
        v, it, reset, _, session, lhash, _ = self.slot.read_header()
        if session != self.slot.session or lhash != self.slot.layout_hash or self.slot.replaced() or \
                not self.slot.owner_alive():
            self.stale = True                 # another publisher owns the path now: re-attach (actor/comm.py)
            return False
        if v % 2 or v == self.version:
            return False
        self.flat_dev.copy_(self.slot.payload, non_blocking=True)
        if self.device.type == 'cuda':
            torch.cuda.current_stream(self.device).synchronize()
        if self.slot.read_header()[0] != v:
            return False                      # torn: a publish started meanwhile; the next poll takes it
        with torch.no_grad():
            _copy_many(self._dsts, self._srcs)
        self.version, self.last_iter, self.reset_flag = v, it, bool(reset)
        return True

    def close(self) -> None:
        self.slot.close()
