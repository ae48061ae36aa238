"""Bucketed gradient all-reduce: multi-process gloo (world 2) on CPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.parallel.dp import GradientReducer
    pdist.init(backend='gloo')
    torch.manual_seed(rank)  # different init per rank -> broadcast must fix it
    m = torch.nn.Sequential(torch.nn.Linear(7, 33), torch.nn.ReLU(), torch.nn.Conv1d(33, 5, 1) if False else torch.nn.Linear(33, 5))
    conv = torch.nn.Conv2d(3, 4, 3).to(memory_format=torch.channels_last)
    params = list(m.parameters()) + list(conv.parameters())
    pdist.broadcast_tensors([p.data for p in params])
    red = GradientReducer(params, bucket_mb=0.0005)  # tiny buckets -> several buckets
    for step in range(2):
        red.zero_grad()
        x = torch.randn(4, 7) * (rank + 1)
        img = torch.randn(2, 3, 6, 6).contiguous(memory_format=torch.channels_last) * (rank + 1)
        (m(x).square().sum() + conv(img).sum()).backward()
        red.synchronize()
    grads = [p.grad.clone() for p in params]
    sc = {k: float(v) for k, v in pdist.allreduce_scalars({'a': torch.tensor(float(rank)), 'b': torch.tensor(2.0)}).items()}
    q.put((rank, [g.numpy() for g in grads], [p.data.clone().numpy() for p in params], sc, red.num_buckets,
           [p.grad.stride() == p.stride() for p in params]))
    pdist.finalize()


def test_gradient_reducer_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    (_, g0, p0, sc0, nb, strides_ok), (_, g1, p1, sc1, _, _) = res
    assert nb > 1
    assert all(strides_ok)
    for a, b in zip(p0, p1):
        assert (a == b).all()             # broadcast made parameters identical
    for a, b in zip(g0, g1):
        assert np.allclose(a, b)          # all-reduced gradients identical on both ranks
    assert sc0 == sc1 and abs(sc0['a'] - 0.5) < 1e-6 and abs(sc0['b'] - 2.0) < 1e-6


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = torch.nn.Linear(6, 16)
        self.ln = torch.nn.LayerNorm(16)
        self.fc2 = torch.nn.Linear(16, 3)
        self.conv = torch.nn.Conv2d(2, 4, 3)

    def forward(self, x, img):
        return self.fc2(torch.relu(self.ln(self.fc1(x)))).square().sum() + self.conv(img).square().sum()


def _master_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.parallel.mixed import MasterWeights
    pdist.init(backend='gloo')
    torch.manual_seed(0)
    m = _Tiny()
    m.conv.to(memory_format=torch.channels_last)
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    mw = MasterWeights(m, bucket_mb=0.0005)
    opt = torch.optim.SGD(mw.opt_params, lr=0.1)
    torch.manual_seed(100 + rank)
    x, img = torch.randn(5, 6), torch.randn(2, 2, 5, 5).contiguous(memory_format=torch.channels_last)
    mw.zero_grad()
    with torch.autocast('cpu', dtype=torch.bfloat16):
        loss = m(x, img)
    loss.backward()
    mw.synchronize()
    opt.step()
    mw.after_step()
    npy = lambda d: {k: v.detach().float().numpy().copy() for k, v in d.items()}  # plain pickles
    q.put((rank, npy(mw.state_dict()), npy(ref), [str(b.flat.dtype) for b in mw.reducer.buckets],
           str(m.fc1.weight.dtype), str(m.ln.weight.dtype), {k: str(v.dtype) for k, v in mw.state_dict().items()}))
    pdist.finalize()


def test_master_weights_world2():
    """bf16 compute weights + flat fp32 masters: masters stay identical across ranks, updates use the
    rank-averaged gradient, norm params stay fp32, bf16 and fp32 params get separate bucket chains."""
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_master_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    import numpy as np
    (_, s0, ref, dts, wdt, lndt, sdt), (_, s1, _, _, _, _, _) = res
    assert wdt == 'torch.bfloat16' and lndt == 'torch.float32'
    assert 'torch.bfloat16' in dts and 'torch.float32' in dts
    assert all(v == 'torch.float32' for v in sdt.values())   # checkpoints carry fp32 masters
    for k in s0:
        assert np.array_equal(s0[k], s1[k]), k
    # the update moved every weight by lr * averaged grad (non-zero)
    assert all(np.abs(s0[k] - ref[k]).max() > 0 for k in ('fc1.weight', 'fc2.weight', 'conv.weight', 'ln.weight'))


def _overlap_worker(rank, world, port, q, defer=False):
    """MasterWeights.backward + synchronize at world 2 (autograd.grad, one copy into the fp32 master gradient,
    flat all-reduce); compared with the average of both ranks' gradients computed locally."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.parallel.mixed import MasterWeights
    pdist.init(backend='gloo')
    torch.manual_seed(0)
    m = _Tiny()
    m.unused = torch.nn.Linear(4, 4)           # a bucket-mate that gets no gradient
    m.conv.to(memory_format=torch.channels_last)
    mw = MasterWeights(m, bucket_mb=0.0002)
    mw.defer_allreduce = defer

    def data(r):
        g = torch.Generator().manual_seed(100 + r)
        return torch.randn(5, 6, generator=g), torch.randn(2, 2, 5, 5, generator=g).contiguous(
            memory_format=torch.channels_last)

    def loss_of(r):
        x, img = data(r)
        with torch.autocast('cpu', dtype=torch.bfloat16):
            return m(x, img)

    # reference: both ranks' gradients on this process, averaged in fp32 (master order via the views)
    ref = {}
    for r in range(world):
        gs = torch.autograd.grad(loss_of(r), mw.reducer.params, allow_unused=True)
        for p, g in zip(mw.reducer.params, gs):
            g = torch.zeros_like(p, dtype=torch.float32) if g is None else g.float()
            ref[p] = ref.get(p, 0) + g / world
    results = []
    for step in range(2):                        # twice: buffers are fully rewritten each step
        mw.zero_grad()
        mw.backward(loss_of(rank))
        mw.synchronize()
        views = mw._master_grad_views()
        results.append(max(float((views.get(p, p.grad).float() - ref[p]).abs().max()) for p in mw.reducer.params))
    nb = mw.reducer.num_buckets
    q.put((rank, results, nb, float(views[m.unused.weight].abs().max())))
    pdist.finalize()


@pytest.mark.parametrize('defer', [False, True])
def test_master_weights_overlapped_backward_world2(defer):
    """Both settings of ``defer_allreduce`` (the eager step and the graph-captured step's contract) take the
    same path: backward writes the local gradient, synchronize() reduces the flat master gradient; the
    unused bucket-mate ends with an exact zero gradient."""
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, q, defer)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, errs, nb, unused in res:
        assert nb > 2
        assert all(e < 1e-5 for e in errs), (rank, errs)
        assert unused == 0.0


def _distmodule_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.parallel.dist_module import DistModule
    pdist.init_from_method('single_node', port=port, backend='gloo')
    torch.manual_seed(rank)
    dm = DistModule(_Tiny(), bucket_mb=0.0005)
    torch.manual_seed(200 + rank)
    x, img = torch.randn(5, 6), torch.randn(2, 2, 5, 5)
    dm.zero_grad()
    dm(x, img).backward()
    dm.sync_gradients()
    # single-process reference: mean of the two ranks' gradients on the same (broadcast) weights
    ref = _Tiny()
    ref.load_state_dict(dm.state_dict())
    tot = [torch.zeros_like(p) for p in ref.parameters()]
    for r in range(world):
        torch.manual_seed(200 + r)
        xr, ir = torch.randn(5, 6), torch.randn(2, 2, 5, 5)
        ref.zero_grad()
        ref(xr, ir).backward()
        tot = [t + p.grad / world for t, p in zip(tot, ref.parameters())]
    ok = all(torch.allclose(p.grad, t, atol=1e-5) for p, t in zip(dm.parameters(), tot))
    grp = pdist.get_group(1)  # world split into singleton groups
    v = torch.tensor([float(rank + 1)])
    pdist.allreduce(v, group=grp)   # singleton group: unchanged
    w = torch.tensor([float(rank + 1)])
    pdist.allreduce(w)              # world: mean 1.5
    q.put((rank, ok, list(dm.state_dict())[:2], float(v), float(w), pdist._slurm_master('gpu[07-09,12],x')))
    pdist.finalize()


def test_dist_module_and_groups_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_distmodule_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    for rank, ok, keys, v, w, master in res:
        assert ok
        assert keys == ['fc1.weight', 'fc1.bias']
        assert v == rank + 1 and abs(w - 1.5) < 1e-6
        assert master == 'gpu07'
