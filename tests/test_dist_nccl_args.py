"""The RCCL-only branches of the data-parallel stack, checked on the CPU by recording the arguments they pass
to torch.distributed (they run for real only on a multi-GPU node): ``init_process_group(device_id=...)`` for the
nccl backend, ``barrier(device_ids=[...])``, ``ReduceOp.AVG`` inside RCCL for bucket / master / scalar
reductions (SUM + divide on gloo), and the health gate's MIN reduction (runtime/train_engine.py)."""
import types

import pytest
import torch
import torch.distributed as dist

from applestar_amd.parallel import dist as pdist


class _Rec:
    def __init__(self, backend='nccl', world=4):
        self.backend, self.world, self.calls = backend, world, []

    def install(self, mp):
        mp.setattr(dist, 'is_available', lambda: True)
        mp.setattr(dist, 'is_initialized', lambda: True)
        mp.setattr(dist, 'get_world_size', lambda group=None: self.world)
        mp.setattr(dist, 'get_rank', lambda group=None: 0)
        mp.setattr(dist, 'get_backend', lambda group=None: self.backend)

        class _H:
            def wait(self_inner):
                return None

        def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
            self.calls.append(('all_reduce', op, tuple(t.shape), t.dtype))
            return _H() if async_op else None

        def barrier(group=None, device_ids=None, **kw):
            self.calls.append(('barrier', device_ids))
        mp.setattr(dist, 'all_reduce', all_reduce)
        mp.setattr(dist, 'barrier', barrier)


def test_init_process_group_passes_device_id_for_nccl(monkeypatch):
    got = {}
    monkeypatch.setattr(dist, 'is_initialized', lambda: False)
    monkeypatch.setattr(dist, 'init_process_group', lambda **kw: got.update(kw))
    monkeypatch.setattr(torch.cuda, 'is_available', lambda: True)
    monkeypatch.setattr(torch.cuda, 'device_count', lambda: 8)
    monkeypatch.setattr(torch.cuda, 'set_device', lambda d: got.setdefault('set_device', d))
    monkeypatch.setattr(torch.cuda, 'current_device', lambda: 3)
    monkeypatch.setenv('WORLD_SIZE', '8')
    monkeypatch.setenv('RANK', '3')
    monkeypatch.setenv('LOCAL_RANK', '3')
    monkeypatch.delenv('APPLESTAR_DIST_BACKEND', raising=False)
    assert pdist.init() == (3, 8)
    assert got['backend'] == 'nccl' and got['device_id'] == torch.device('cuda', 3) and got['set_device'] == 3
    got.clear()
    monkeypatch.setenv('APPLESTAR_DIST_BACKEND', 'gloo')          # one-GPU rehearsal: no device_id for gloo
    pdist.init()
    assert got['backend'] == 'gloo' and 'device_id' not in got


@pytest.mark.parametrize('backend', ['nccl', 'gloo'])
def test_reductions_use_avg_only_on_rccl(monkeypatch, backend):
    rec = _Rec(backend)
    rec.install(monkeypatch)
    monkeypatch.setattr(torch.cuda, 'current_device', lambda: 5)
    pdist.barrier()
    assert rec.calls[-1] == ('barrier', [5] if backend == 'nccl' else None)
    from applestar_amd.parallel.dp import GradientReducer
    ps = [torch.nn.Parameter(torch.randn(10, 3)), torch.nn.Parameter(torch.randn(7))]
    red = GradientReducer(ps, bucket_mb=32)
    for p in ps:
        p.grad.fill_(4.0)
    red.synchronize()
    ops = [c[1] for c in rec.calls if c[0] == 'all_reduce']
    assert ops and all(op == (dist.ReduceOp.AVG if backend == 'nccl' else dist.ReduceOp.SUM) for op in ops)
    # gloo: SUM then divide by the world size (the recorded collective did not touch the data)
    expect = 4.0 if backend == 'nccl' else 1.0
    assert all(torch.all(p.grad == expect) for p in ps)
    x = torch.ones(3)
    pdist.allreduce(x)
    assert rec.calls[-1][1] == (dist.ReduceOp.AVG if backend == 'nccl' else dist.ReduceOp.SUM)


def test_health_gate_min_reduced_with_the_buckets(monkeypatch):
    """TrainEngine._reduce: the LSTM health gate goes through a MIN all-reduce before the update on every rank."""
    from applestar_amd.runtime.train_engine import TrainEngine
    rec = _Rec('nccl', world=2)
    rec.install(monkeypatch)
    eng = TrainEngine.__new__(TrainEngine)
    eng.device = torch.device('cpu')
    eng._gate = torch.ones(())
    eng.master = None
    eng.reducer = types.SimpleNamespace(synchronize=lambda: rec.calls.append(('buckets',)))
    eng._lstm_gate = lambda: torch.zeros(())
    eng._reduce()
    assert ('all_reduce', dist.ReduceOp.MIN, (), torch.float32) in rec.calls
    assert rec.calls.index(('buckets',)) > [i for i, c in enumerate(rec.calls) if c[0] == 'all_reduce'][0]
    assert float(eng._gate) == 0.0
