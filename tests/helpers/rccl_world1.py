"""Child script of tests/test_dist_rccl_gpu.py: the nccl (RCCL) branches of parallel/dist.py and parallel/dp.py
on a real GPU at world size 1 (one GPU per rank is all a 1-GPU box can host: RCCL refuses two ranks on one
device, "Duplicate GPU detected").  Prints one JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from applestar_amd.parallel import dist as pdist
    from applestar_amd.parallel.dp import GradientReducer
    port = int(sys.argv[1])
    rank, world = pdist.init(init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1, timeout_s=120)
    dev = torch.device('cuda', torch.cuda.current_device())
    rec = {'backend': dist.get_backend(), 'world': world, 'device': str(dev)}
    pdist.barrier()                                            # nccl: barrier(device_ids=[...])
    x = torch.arange(8, dtype=torch.float32, device=dev)
    dist.all_reduce(x, op=dist.ReduceOp.AVG)                   # the AVG op GradientReducer uses on nccl
    rec['avg_ok'] = bool(torch.equal(x, torch.arange(8, dtype=torch.float32, device=dev)))
    g = torch.ones((), device=dev)
    dist.all_reduce(g, op=dist.ReduceOp.MIN)                   # the LSTM health gate's MIN reduction
    rec['min_ok'] = float(g) == 1.0
    out = [torch.zeros(4, device=dev)]
    dist.all_gather(out, torch.full((4,), 3.0, device=dev))   # bench.py's replica check
    rec['all_gather_ok'] = bool(torch.all(out[0] == 3.0))
    b = torch.randn(5, device=dev)
    b0 = b.clone()
    dist.broadcast(b, 0)
    rec['broadcast_ok'] = bool(torch.equal(b, b0))
    # the bucketed reducer's RCCL path: flat buckets, one async AVG all-reduce per bucket, wait - forced on at
    # world 1 (an average over one rank is the identity, so the buckets must come back bit-identical)
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 32)).to(dev)
    red = GradientReducer(list(net.parameters()), bucket_mb=0.05)
    red.world, red.use_avg = 2, True
    red.backward(net(torch.randn(16, 64, device=dev)).square().sum())
    ref = [p.grad.clone() for p in net.parameters()]
    red.synchronize()
    torch.cuda.synchronize()
    rec['reducer_buckets'] = red.num_buckets
    rec['reducer_ok'] = all(torch.equal(p.grad, r) for p, r in zip(net.parameters(), ref))
    pdist.finalize()
    print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
