"""Bucketed gradient all-reduce: multi-process gloo (world 2) on CPU."""
import os
import socket

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
    sc = pdist.allreduce_scalars({'a': torch.tensor(float(rank)), 'b': torch.tensor(2.0)})
    q.put((rank, [g for g in grads], [p.data.clone() for p in params], sc, red.num_buckets,
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
        assert torch.equal(a, b)          # broadcast made parameters identical
    for a, b in zip(g0, g1):
        assert torch.allclose(a, b)       # all-reduced gradients identical on both ranks
    assert sc0 == sc1 and abs(sc0['a'] - 0.5) < 1e-6 and abs(sc0['b'] - 2.0) < 1e-6
