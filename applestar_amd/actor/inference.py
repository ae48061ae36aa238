"""Batched GPU inference server for actors (the reference's ``gpu_batch_inference``).

Reference (``agent.py:145-158,364-385,781-805``, ``actor.py:268-299``): every env process writes its
observation into a shared-memory slot and bumps a signal; a GPU loop runs ``compute_logp_action`` on
*all* slots (active or not) and copies flagged rows back; env processes poll with ``sleep(0.01)``; the teacher
forward of ``collect_data`` is a second, separate model call per agent step.

MI355X design:
* one server per GPU owns every model (policy per player, teacher per player) on the device;
* env workers send one request frame (``utils.serialize``, native codec) over a pipe and block on the reply -
  no polling.  Each pipe is bound to a ROUTE ``(player, kind, teacher)`` when it is registered, so the server
  never decodes a request on its own: B frames go straight into ``collate_frames`` (csrc/codec.cpp), which
  lays the collated batch out in ONE pinned staging buffer (entities padded to the batch's entity BUCKET,
  128 / 256 / 512) that is copied with one H2D DMA;
* ``kind='policy+teacher'`` serves a training agent's step in ONE request: the policy samples the action and
  the teacher's teacher-forced logits for that very action are computed in the same HIP graph (the
  reference's two round trips per agent step become one; ``agent.py`` caches the teacher half for
  ``collect_data``);
* every (route, batch bucket, entity bucket) is a captured HIP graph (``runtime.graphs.GraphedPolicy``);
* two-stage pipeline: a batch is LAUNCHED (H2D, replay, async D2H into pinned memory, event) and FINISHED
  (event wait, per-row replies) on the next loop turn, after the next batch was collected and launched -
  the host work of batch k+1 overlaps the GPU work of batch k, and replies go out as soon as the event fired.
"""
from __future__ import annotations

import os
import threading
import time
from collections import defaultdict, deque
from multiprocessing.connection import Connection, wait
from typing import Dict, List, Optional, Tuple

import torch

from ..agent.collate import collate_obs, decollate_output
from ..utils import serialize

ENTITY_BUCKETS = (128, 256, 512)
POLICY_TEACHER = 'policy+teacher'


def _to(tree, device, non_blocking=True):
    if isinstance(tree, torch.Tensor):
        if device.type == 'cuda':
            return tree.pin_memory().to(device, non_blocking=non_blocking)
        return tree
    if isinstance(tree, dict):
        return {k: _to(v, device, non_blocking) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        return type(tree)(_to(v, device, non_blocking) for v in tree)
    return tree



def _refresh_forms(model):
    """New weights are in ``model``'s parameters: rebuild its cached inference weight forms in place (the HIP
    graphs that captured them read the same buffers)."""
    reg = getattr(model, '_inference_forms', None)
    if reg is not None:
        with torch.no_grad():
            reg.refresh()

class InferenceClient:
    """Worker-side handle: ``infer(model_input) -> per-sample output`` (blocking).  The connection is bound to
    its route on the server side (``InferenceServer.add_connection(conn, route)``), so a request is the bare
    model input; routes registered without a key get the self-describing envelope."""

    def __init__(self, conn: Connection, player_id: str, kind: str = 'policy', teacher_id: Optional[str] = None,
                 routed: bool = True):
        self._conn = conn
        self.player_id = player_id
        self.kind = kind
        self.teacher_id = teacher_id
        self.routed = routed

    def infer(self, model_input: Dict) -> Dict:
        if self.routed:
            self._conn.send_bytes(serialize.dumps(model_input))
        else:
            self._conn.send_bytes(serialize.dumps({'player_id': self.player_id, 'kind': self.kind,
                                                   'teacher_id': self.teacher_id, 'input': model_input}))
        return serialize.loads(self._conn.recv_bytes())


class _PolicyTeacher(torch.nn.Module):
    """One agent step of a training actor: policy sample + the teacher's logits for the sampled action
    (``compute_logp_action`` then ``compute_teacher_logit`` with the teacher's own LSTM state)."""

    def __init__(self, policy, teacher):
        super().__init__()
        self.policy, self.teacher = policy, teacher

    def step(self, spatial_info, entity_info, scalar_info, entity_num, hidden_state, teacher_hidden_state,
             noise=None, **kwargs):
        out = self.policy.compute_logp_action(spatial_info, entity_info, scalar_info, entity_num, hidden_state,
                                              noise=noise)
        t = self.teacher.compute_teacher_logit(spatial_info, entity_info, scalar_info, entity_num,
                                               teacher_hidden_state, out['selected_units_num'], out['action_info'])
        out['teacher'] = {'logit': t['logit'], 'hidden_state': t['hidden_state']}
        return out


class _Launched:
    __slots__ = ('conns', 'n', 'out', 'event', 'route', 'keep_logits', 't0')


class InferenceServer:
    def __init__(self, device='cuda', max_wait_ms: float = 2.0, amp_dtype: Optional[torch.dtype] = torch.bfloat16,
                 use_graphs: Optional[bool] = None, entity_buckets=ENTITY_BUCKETS, max_batch: int = 64):
        self.device = torch.device(device)
        # HIP-graph replay per (route, batch bucket, entity bucket); a handful of captured graphs serve every request
        self.use_graphs = (self.device.type == 'cuda' and amp_dtype == torch.bfloat16) if use_graphs is None \
            else bool(use_graphs)
        self.entity_buckets = tuple(sorted(entity_buckets))
        self.max_batch = int(max_batch)
        self._graphed: Dict[tuple, object] = {}
        self._runners: Dict[tuple, torch.nn.Module] = {}
        self.max_wait = max_wait_ms / 1000.0
        self.max_busy_wait = 0.05       # cap on collecting behind an in-flight batch (seconds)
        self.amp_dtype = amp_dtype if self.device.type == 'cuda' else None
        # the server's device work (H2D, graph replays, D2H) on a HIGH-priority stream: on a GPU shared with the
        # learner, the dispatcher starts the actors' small inference kernels ahead of the learner's queued
        # workgroups, so the agent-step round trip does not wait behind a learner step
        # (APPLESTAR_INFERENCE_STREAM_PRIORITY=0: the default stream)
        prio = int(os.environ.get('APPLESTAR_INFERENCE_STREAM_PRIORITY', '-1'))
        self._stream = torch.cuda.Stream(device=self.device, priority=prio) \
            if self.device.type == 'cuda' and prio != 0 else None
        self.models: Dict[str, torch.nn.Module] = {}
        self.teachers: Dict[str, torch.nn.Module] = {}
        self.model_iter: Dict[str, int] = defaultdict(int)
        self._conns: List[Connection] = []
        self._routes: Dict[Connection, Optional[tuple]] = {}
        self._lock = threading.Lock()
        self._stop = False
        self._inflight: deque = deque()
        self.stats = defaultdict(float)

    # ------------------------------------------------------------------ models
    def set_model(self, player_id: str, model: torch.nn.Module, teacher: bool = False):
        model = model.to(self.device).eval()
        if self.device.type == 'cuda' and getattr(model, '_inference_forms', None) is None:
            # bf16 / transposed weight forms cast once per weight version, not inside every graph replay
            from ..ops import native
            if native.ensure_loaded() is not None:
                model._inference_forms = native.attach_inference_forms(model)
        with self._lock:
            (self.teachers if teacher else self.models)[player_id] = model
            self._graphed = {k: v for k, v in self._graphed.items() if player_id not in k[0][::2]}
            self._runners = {k: v for k, v in self._runners.items() if player_id not in k[::2]}

    def load_state_dict(self, player_id: str, state_dict: Dict, teacher: bool = False, last_iter: int = 0):
        """Hot model update (weights pulled from the learner) without rebuilding the module.  Captured graphs
        stay valid: they read the parameters in place and recompute every weight-derived table inside the graph
        (models/heads.py ``_capturing``)."""
        with self._lock:
            m = (self.teachers if teacher else self.models)[player_id]
            own = m.state_dict()
            self._weights_begin()
            with torch.no_grad():
                for k, v in state_dict.items():
                    if k in own and own[k].shape == v.shape:
                        own[k].copy_(v, non_blocking=True)
            _refresh_forms(m)
            self._weights_end()
            if not teacher:
                self.model_iter[player_id] = int(last_iter)

    def load_flat(self, player_id: str, flat: torch.Tensor, names, shapes, last_iter: int = 0):
        """Hot update from the learner's flat snapshot (runtime/flat_model.py): ONE H2D copy of the flat vector,
        then ONE native multi-tensor D2D copy into the resident model's tensors."""
        from ..runtime.flat_model import _copy_many
        with self._lock:
            m = self.models[player_id]
            own = m.state_dict()
            dev = next(m.parameters()).device
            flat_dev = flat.to(dev, non_blocking=True)
            dsts, srcs, off = [], [], 0
            for k, shp in zip(names, shapes):
                n = 1
                for d in shp:
                    n *= int(d)
                t = own.get(k)
                if t is not None and tuple(t.shape) == tuple(shp) and t.dtype == torch.float32:
                    dsts.append(t)
                    srcs.append(flat_dev[off:off + n].view(tuple(shp)))
                off += n
            self._weights_begin()
            with torch.no_grad():
                _copy_many(dsts, srcs)
            _refresh_forms(m)
            self._weights_end()
            self.model_iter[player_id] = int(last_iter)

    def attach_model_slot(self, player_id: str, shm_name: str) -> bool:
        """Co-located learner: read ``player_id``'s published policy straight from its /dev/shm slot (seqlock
        version, one H2D + one D2D multi-copy per new version; runtime/flat_model.ModelSubscriber)."""
        import os
        from ..runtime.flat_model import FlatLayout, ModelSubscriber
        if not os.path.exists(os.path.join('/dev/shm', shm_name)):
            return False
        with self._lock:
            m = self.models[player_id]
            sub = ModelSubscriber(m, shm_name)
            sd = m.policy_state_dict() if hasattr(m, 'policy_state_dict') else m.state_dict()
            layout = FlatLayout({k: v for k, v in sd.items() if v.dtype == torch.float32})
            try:
                sub.bind(layout)           # element count AND the (name, shape) hash the publisher stamped
            except ValueError:
                sub.close()
                return False
            if sub.stale:                  # left behind by a learner that exited: not this run's weights
                sub.close()
                return False
            self._subscribers = getattr(self, '_subscribers', {})
            old = self._subscribers.pop(player_id, None)
            if old is not None:
                old.close()
            self._subscribers[player_id] = sub
        return True

    def detach_model_slot(self, player_id: str) -> None:
        """Stop reading ``player_id``'s slot (it went stale, or the network broadcast overtook it)."""
        with self._lock:
            sub = getattr(self, '_subscribers', {}).pop(player_id, None)
        if sub is not None:
            sub.close()

    def model_slot_state(self, player_id: str) -> Optional[str]:
        """None (not attached), 'live' or 'stale' (the path now names another publisher's slot)."""
        sub = getattr(self, '_subscribers', {}).get(player_id)
        return None if sub is None else ('stale' if sub.stale else 'live')

    def poll_model_slots(self) -> Dict[str, int]:
        """Apply any newer published versions; returns {player_id: model_last_iter} of the updated ones."""
        out = {}
        for pid, sub in list(getattr(self, '_subscribers', {}).items()):
            with self._lock:
                self._weights_begin()
                updated = sub.poll()
                if updated:
                    _refresh_forms(self.models[pid])
                self._weights_end()
                if updated:
                    self.model_iter[pid] = sub.last_iter
                    out[pid] = sub.last_iter
        return out

    def add_connection(self, conn: Connection, route: Optional[Tuple[str, str, Optional[str]]] = None):
        """``route`` = (player_id, kind, teacher_id): requests on ``conn`` are bare model inputs for that route
        (kind 'policy', 'teacher' or 'policy+teacher'); None: self-describing envelopes."""
        with self._lock:
            self._conns.append(conn)
            self._routes[conn] = tuple(route) if route is not None else None

    # ------------------------------------------------------------------ execution
    def _runner(self, route) -> Tuple[torch.nn.Module, str]:
        pid, kind, tid = route
        with self._lock:
            if kind == 'policy':
                return self.models[pid], 'compute_logp_action'
            if kind == 'teacher':
                return self.teachers[pid], 'compute_teacher_logit'
            r = self._runners.get(route)
            if r is None:
                r = self._runners[route] = _PolicyTeacher(self.models[pid], self.teachers[tid or pid])
            return r, 'step'

    def _bucket(self, n: int) -> int:
        for b in self.entity_buckets:
            if b >= n:
                return b
        return n

    def _collate(self, frames: List[bytes], inputs: Optional[List[Dict]], rows: int, graphs: bool):
        """Device batch of ``rows`` samples (dummy copies of sample 0 pad a graph's batch bucket)."""
        from ..ops import _ext
        nat = _ext._load()
        if frames is not None and nat is not None and hasattr(nat, 'collate_frames'):
            fr = list(frames) + [frames[0]] * (rows - len(frames))
            dev = self.device if self.device.type == 'cuda' else None
            return nat.collate_frames(fr, 0, None if dev is None else str(dev),
                                      list(self.entity_buckets) if graphs else [])
        if inputs is None:
            inputs = [serialize.loads(f) for f in frames]
        inputs = list(inputs) + [inputs[0]] * (rows - len(inputs))
        pad = self._bucket(max(int(o['entity_num']) for o in inputs)) if graphs else 0
        batch = collate_obs(inputs, pad_entities=pad)
        return _packed_to(batch, self.device)

    def _launch(self, route, frames=None, inputs=None, keep_logits: bool = False) -> _Launched:
        t0 = time.perf_counter()
        model, method = self._runner(route)
        n = len(frames) if frames is not None else len(inputs)
        graphs = self.use_graphs
        rows = 1 << (n - 1).bit_length() if graphs else n            # batch bucket (power of two)
        batch = self._collate(frames, inputs, rows, graphs)
        t1 = time.perf_counter()
        self.stats['collate_h2d_s'] += t1 - t0
        if graphs:
            from ..runtime.graphs import GraphedPolicy
            key = (route, rows, batch['entity_info']['unit_type'].shape[-1])
            gp = self._graphed.get(key)
            if gp is None:
                gp = self._graphed[key] = GraphedPolicy(model, method, max_graphs=1)
            out = gp(**batch)
        else:
            ctx = torch.autocast('cuda', dtype=self.amp_dtype) if self.amp_dtype else _null()
            with torch.no_grad(), ctx:
                out = getattr(model, method)(**batch)
        self.stats['launch_s'] += time.perf_counter() - t1
        if not keep_logits and route[1] != 'teacher':
            out = {k: v for k, v in out.items() if k != 'logit'}     # the agent keeps only the taken action's logp
        L = _Launched()
        L.n, L.route, L.keep_logits, L.t0 = n, route, keep_logits, t0
        L.out = _to_cpu_async(out)        # pinned, non_blocking: copied before the next replay overwrites them
        L.event = None
        if self.device.type == 'cuda':
            L.event = torch.cuda.Event()
            L.event.record()
        return L

    def _wait(self, L: _Launched) -> float:
        t0 = time.perf_counter()
        if L.event is not None:
            L.event.synchronize()
        t1 = time.perf_counter()
        self.stats['d2h_wait_s'] += t1 - t0
        return t1

    def _reply_frames(self, L: _Launched) -> Optional[List[bytes]]:
        """Per-row reply frames straight from the host batch (csrc/codec.cpp rows_dumps: decollate_output's
        trimming and the encode in one native pass); None without the extension."""
        from ..ops import _ext
        nat = _ext._load()
        if nat is None or not hasattr(nat, 'rows_dumps'):
            return None
        t1 = self._wait(L)
        out = dict(L.out)
        n = L.n
        s = [int(v) for v in out['selected_units_num'][:n].tolist()]
        e = [int(v) for v in out['entity_num'][:n].tolist()]
        e1 = [v + 1 for v in e]
        trims = {'logit/selected_units': [(0, s), (1, e1)], 'logit/target_unit': [(0, e)],
                 'action_info/selected_units': [(0, s)], 'action_logp/selected_units': [(0, s)],
                 'extra_units': [(0, e)],
                 'teacher/logit/selected_units': [(0, s), (1, e1)], 'teacher/logit/target_unit': [(0, e)]}
        pid, kind, _ = L.route
        if kind != 'teacher':
            out['model_last_iter'] = self.model_iter[pid]
        frames = nat.rows_dumps(out, n, trims)
        self.stats['decollate_s'] += time.perf_counter() - t1
        return frames

    def _results(self, L: _Launched) -> List[Dict]:
        t1 = self._wait(L)
        out = L.out
        teacher = out.pop('teacher', None)
        res = [decollate_output(out, i) for i in range(L.n)]
        if teacher is not None:
            t = dict(teacher, entity_num=out['entity_num'], selected_units_num=out['selected_units_num'])
            for i, r in enumerate(res):
                td = decollate_output(t, i)
                r['teacher'] = {'logit': td['logit'], 'hidden_state': td['hidden_state']}
        pid, kind, _ = L.route
        if kind != 'teacher':
            for r in res:
                r['model_last_iter'] = self.model_iter[pid]
        self.stats['decollate_s'] += time.perf_counter() - t1
        return res

    def _on_stream(self):
        return torch.cuda.stream(self._stream) if self._stream is not None else _null()

    def _weights_begin(self):
        """Before writing a model's weights (any thread): the server's queued work that reads them goes first."""
        if self._stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._stream)

    def _weights_end(self):
        """After writing: the server's later work waits for the writes."""
        if self._stream is not None:
            self._stream.wait_stream(torch.cuda.current_stream(self.device))

    def _forward(self, player_id: str, kind: str, inputs: List[Dict], teacher_id: Optional[str] = None) -> List[Dict]:
        """Synchronous batch of decoded inputs (tests / in-process callers); replies keep the policy logits."""
        with self._on_stream():
            return self._results(self._launch((player_id, kind, teacher_id), inputs=inputs, keep_logits=True))

    # ------------------------------------------------------------------ serving
    def _finish(self, L: _Launched):
        frames = self._reply_frames(L)
        if frames is None:
            frames = [serialize.dumps(o) for o in self._results(L)]
        t0 = time.perf_counter()
        for c, f in zip(L.conns, frames):
            try:
                c.send_bytes(f)
            except (BrokenPipeError, OSError):
                pass
        self.stats['reply_s'] += time.perf_counter() - t0
        self.stats['served_s'] += time.perf_counter() - L.t0

    def _collect(self, timeout: float, busy=None) -> Dict[tuple, List[Tuple[Connection, bytes]]]:
        """Requests that arrived.  ``busy``: the GPU is still running the in-flight batch - keep collecting
        (the next batch could not start earlier anyway) until it finishes, every live pipe has asked, or
        ``max_busy_wait`` passed: under load the batches grow by themselves, which makes every row cheaper."""
        with self._lock:
            conns = list(self._conns)
        groups: Dict[tuple, List] = defaultdict(list)
        if not conns:
            if timeout > 0:
                time.sleep(timeout)
            return groups
        pending: Dict[Connection, bytes] = {}
        if busy is not None:
            t_end = time.time() + self.max_busy_wait
            while busy() and len(pending) < len(self._conns) and time.time() < t_end:
                for c in wait([c for c in conns if c not in pending and c in self._conns], timeout=0.0005):
                    try:
                        pending[c] = c.recv_bytes()
                    except (EOFError, OSError):
                        with self._lock:
                            if c in self._conns:
                                self._conns.remove(c)
                                self._routes.pop(c, None)
            ready = [c for c in wait([c for c in conns if c not in pending], timeout=0.0)]
        else:
            ready = wait(conns, timeout=timeout)
        if not ready and not pending:
            return groups
        deadline = time.time() + (self.max_wait if timeout > 0 else 0.0)
        while True:
            for c in ready:
                if c in pending:
                    continue
                try:
                    pending[c] = c.recv_bytes()
                except (EOFError, OSError):
                    with self._lock:
                        if c in self._conns:
                            self._conns.remove(c)
                            self._routes.pop(c, None)
            live = len(self._conns)
            left = deadline - time.time()
            if len(pending) >= live or left <= 0:
                break
            ready = [c for c in wait([c for c in conns if c not in pending and c in self._conns], timeout=left)]
            if not ready:
                break
        for c, frame in pending.items():
            route = self._routes.get(c)
            if route is None:                       # envelope: decode to find the route
                req = serialize.loads(frame)
                route = (req['player_id'], req['kind'], req.get('teacher_id'))
                frame = serialize.dumps(req['input'])
            groups[route].append((c, frame))
        return groups

    def serve_once(self, timeout: float = 0.1) -> int:
        """Collect one dynamic batch per route and launch it; finish (reply to) the batches launched on the
        previous call.  Returns the number of requests launched."""
        with self._on_stream():
            return self._serve_once(timeout)

    def _serve_once(self, timeout: float) -> int:
        busy = None
        if self._inflight and self._inflight[-1].event is not None:
            ev = self._inflight[-1].event
            busy = lambda: not ev.query()
        groups = self._collect(0.0 if self._inflight else timeout, busy)
        prev = list(self._inflight)
        self._inflight.clear()
        served = 0
        for route, items in groups.items():
            for s in range(0, len(items), self.max_batch):
                chunk = items[s:s + self.max_batch]
                L = self._launch(route, frames=[f for _, f in chunk])
                L.conns = [c for c, _ in chunk]
                self._inflight.append(L)
                self.stats['batches'] += 1
                served += len(chunk)
        for L in prev:
            self._finish(L)
        self.stats['requests'] += served
        return served

    def drain(self):
        with self._on_stream():
            while self._inflight:
                self._finish(self._inflight.popleft())

    def serve_forever(self, stop_event: Optional[threading.Event] = None):
        while not self._stop and not (stop_event is not None and stop_event.is_set()):
            self.serve_once()
        self.drain()

    def stop(self):
        self._stop = True


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _packed_to(batch, device):
    """Host batch -> device: one pinned buffer, one async copy (CPU: unchanged)."""
    if device.type != 'cuda':
        return batch
    from ..runtime.prefetch import pack_tree
    return pack_tree(batch, pin=True).to_device(device)


def _to_cpu_async(tree):
    """Device outputs -> pinned host tensors with non_blocking copies (the caller waits on an event)."""
    if isinstance(tree, torch.Tensor):
        return tree.detach().to('cpu', non_blocking=tree.is_cuda)
    if isinstance(tree, dict):
        return {k: _to_cpu_async(v) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        return type(tree)(_to_cpu_async(v) for v in tree)
    return tree


def _to_cpu(tree, device=None):
    """Device outputs -> host: every copy non-blocking into pinned memory, then ONE stream synchronize."""
    out = _to_cpu_async(tree)
    if device is not None and device.type == 'cuda':
        torch.cuda.current_stream(device).synchronize()
    return out
