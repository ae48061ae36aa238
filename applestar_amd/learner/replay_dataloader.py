"""Supervised-learning data from replays (``sl_dataloader.py:19-189``, ``replay_actor.py:10-75``).

* replay paths: a directory of ``*.SC2Replay`` or a text file with one path per line, repeated
  ``epochs`` times, sharded by data-parallel rank (``sl_dataloader.py:116-125``); both players of
  every replay are decoded;
* ``num_workers`` spawned decoder processes (each with its own SC2 client) stream trajectories back
  as single serialized buffers;
* remote mode: :class:`ReplayActor` processes on other hosts push trajectories to the coordinator
  token ``sl_traj`` and the loader pulls them instead;
* batching: ``batch_size`` slots, each consuming consecutive ``trajectory_length`` chunks of ONE
  replay so the learner can carry the LSTM state (``new_episodes`` marks a slot's first chunk); a
  short final chunk is padded by repeating its last step with every action mask off;
* the shared batch (``sl_dataloader.py:19-94``): on a GPU a collator process packs every batch into one of
  three pinned shared-memory slabs and the learner copies it to HBM with one async DMA on a side stream
  (``runtime/shared_batch.py``), so collation and the H2D copy overlap the previous step.
"""
from __future__ import annotations

import glob
import multiprocessing as mp
import os
import queue
import random
from typing import Iterator, List, Optional

import torch

from ..agent.collate import collate_obs
from ..utils import serialize

STEP_KEYS = ('spatial_info', 'entity_info', 'scalar_info', 'entity_num', 'action_info', 'action_mask',
             'selected_units_num')


def replay_paths(spec: str, epochs: int = 1, rank: int = 0, world_size: int = 1, seed: int = 0) -> List[str]:
    if os.path.isdir(spec):
        paths = sorted(glob.glob(os.path.join(spec, '**', '*.SC2Replay'), recursive=True))
    else:
        with open(spec) as f:
            paths = [l.strip() for l in f if l.strip()]
    rng = random.Random(seed)
    out = []
    for _ in range(max(1, int(epochs))):
        p = list(paths)
        rng.shuffle(p)
        out += p
    return out[rank::world_size]


def _decode_worker(cfg_dict, jobs, out_q):
    from ..utils.config import AttrDict
    from ..agent.replay_decoder import ReplayDecoder
    torch.set_num_threads(1)
    dec = ReplayDecoder(AttrDict(cfg_dict))
    while True:
        job = jobs.get()
        if job is None:
            break
        path, player = job
        traj = dec.run(path, player)
        if traj:
            out_q.put(serialize.dumps([{k: s[k] for k in STEP_KEYS} for s in traj]))
    dec.close()
    out_q.put(None)


class _SlotAssembler:
    """``batch_size`` slots, each consuming consecutive ``trajectory_length`` chunks of ONE trajectory (the
    learner carries the LSTM state per slot; ``new_episodes`` marks a slot's first chunk); a short final chunk
    is padded by repeating its last step with every action mask off.  Yields collated host batches."""

    def __init__(self, source: Iterator, B: int, T: int):
        self._source, self.B, self.T = source, B, T
        self._slots = [None] * B            # (trajectory, cursor)

    def _chunk(self, b: int):
        new = False
        if self._slots[b] is None or self._slots[b][1] >= len(self._slots[b][0]):
            self._slots[b] = (next(self._source), 0)
            new = True
        traj, cur = self._slots[b]
        steps = traj[cur:cur + self.T]
        self._slots[b] = (traj, cur + self.T)
        n = len(steps)
        if n < self.T:
            pad = dict(steps[-1])
            pad['action_mask'] = {k: torch.zeros_like(v) for k, v in steps[-1]['action_mask'].items()}
            steps = steps + [pad] * (self.T - n)
        return steps, n, new

    def __iter__(self):
        return self

    def __next__(self):
        steps, lens, news = [], [], []
        for b in range(self.B):
            s, n, new = self._chunk(b)
            steps += s
            lens.append(n)
            news.append(new)
        batch = collate_obs(steps)                 # batch-major [B*T], entities padded to the max
        batch['traj_lens'] = lens                  # host lists: ride in the slab layout, never on the device
        batch['new_episodes'] = news
        return batch


def _pull_local(out_q, n_workers: int):
    done = 0
    while done < n_workers:
        item = out_q.get()
        if item is None:
            done += 1
            continue
        yield serialize.loads(item)


def _pull_remote(ip, port):
    from ..comm.adapter import Adapter
    adapter = Adapter(ip, port)
    while True:
        for t in adapter.pull('sl_traj', size=1, block=True):
            yield t


class _CollatorBatches:
    """Picklable batch factory run inside the shared-batch collator process: builds the trajectory source
    there (decode-worker queue, remote coordinator, or a user factory) and assembles batches from it."""

    def __init__(self, B, T, kind, *args):
        self.B, self.T, self.kind, self.args = B, T, kind, args

    def __call__(self):
        if self.kind == 'local':
            src = _pull_local(*self.args)
        elif self.kind == 'remote':
            src = _pull_remote(*self.args)
        else:
            src = iter(self.args[0]())
        return _SlotAssembler(src, self.B, self.T)


class ReplayDataLoader:
    """SL batches from replay trajectories.  On a GPU (or with ``learner.data.shared_batch``) a collator process
    packs each batch into a pinned shared-memory slab and the learner issues one async H2D copy of it
    (runtime/shared_batch.py); otherwise batches are collated in-process.  ``source``: an injected trajectory
    iterator (in-process); ``source_factory``: a picklable callable returning one (usable by the collator)."""

    def __init__(self, cfg, device='cpu', rank: int = 0, world_size: int = 1, source: Optional[Iterator] = None,
                 source_factory=None):
        d = cfg.learner.data
        self.B, self.T = int(d.batch_size), int(d.trajectory_length)
        self.device = torch.device(device)
        self._procs = []
        self._shared = None
        if source is not None:                    # injected trajectory iterator (tests / custom sources)
            spec = None
            src = source
        elif source_factory is not None:
            spec = ('factory', source_factory)
        elif d.get('remote', False):              # replay actors push to the coordinator
            spec = ('remote', cfg.communication.coordinator_ip, cfg.communication.coordinator_port)
        else:
            ctx = mp.get_context('spawn')
            jobs, out = ctx.Queue(), ctx.Queue(maxsize=4 * self.B)
            for p in replay_paths(d.train_data_file, d.get('epochs', 1), rank, world_size):
                for player in (0, 1):
                    jobs.put((p, player))
            n = int(d.get('num_workers', 1))
            for _ in range(n):
                jobs.put(None)
                pr = ctx.Process(target=_decode_worker, args=(dict(cfg), jobs, out), daemon=True)
                pr.start()
                self._procs.append(pr)
            spec = ('local', out, n)
        use_shared = bool(d.get('shared_batch', self.device.type == 'cuda')) and spec is not None
        if use_shared:
            from ..runtime.shared_batch import SharedBatchLoader
            self._shared = SharedBatchLoader(_CollatorBatches(self.B, self.T, *spec), self.device,
                                             n_slabs=int(d.get('shared_slabs', 3)),
                                             slab_bytes=int(d.get('slab_mb', 512)) << 20)
            self._iter = self._shared
        else:
            if spec is not None:
                src = _CollatorBatches(1, 1, *spec)()._source
            self._iter = self._in_process(_SlotAssembler(src, self.B, self.T))

    def _in_process(self, assembler):
        for batch in assembler:
            if self.device.type != 'cpu':
                from ..rl.synthetic import to_device
                batch = to_device(batch, self.device)
            yield batch

    def __iter__(self):
        return self

    def __next__(self):
        return next(self._iter)

    def close(self):
        if self._shared is not None:
            self._shared.close()
        for p in self._procs:
            p.terminate()


class ReplayActor:
    """Remote replay decoding: decode this host's shard of replays and push trajectories to the
    coordinator (``replay_actor.py``)."""

    def __init__(self, cfg, rank: int = 0, world_size: int = 1):
        from ..comm.adapter import Adapter
        from ..agent.replay_decoder import ReplayDecoder
        self.cfg = cfg
        d = cfg.learner.data
        self._paths = replay_paths(d.train_data_file, d.get('epochs', 1), rank, world_size)
        self._adapter = Adapter(cfg.communication.coordinator_ip, cfg.communication.coordinator_port)
        self._decoder = ReplayDecoder(cfg)

    def run(self):
        for p in self._paths:
            for player in (0, 1):
                traj = self._decoder.run(p, player)
                if traj:
                    self._adapter.push([{k: s[k] for k in STEP_KEYS} for s in traj], 'sl_traj')
        self._decoder.close()
