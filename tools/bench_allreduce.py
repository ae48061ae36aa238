"""RCCL all-reduce bandwidth for the learner's gradient buckets, one process per GPU (for an 8-GPU node).

    torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py
    torchrun ... tools/bench_allreduce.py --sizes-mb 4,32,132 --dtype float32 --iters 20

For each message size: the time of one in-place ``all_reduce`` (max over ranks, median over iterations,
AVG op inside RCCL) and the ring bus bandwidth 2 (n-1)/n * bytes / time, which on an xGMI-connected MI355X
node is bounded per link (7 links x ~153 GB/s per GPU).  The learner's reduction is ~132 MB of fp32
gradients per step (33 M parameters; parallel/dp.py): the ``--sizes-mb`` default covers the bucket sizes
(32 MB), the whole master gradient (132 MB) and small messages.  Also times the learner's exact call pattern
(``MasterWeights.reduce_flat``-style: one flat fp32 buffer + one small fp32 buffer, async then waited).
Prints one JSON line per size on rank 0.  Not run by the test-suite (needs >= 2 GPUs); the gloo path of the
same code is covered by tests/test_dp_trainer.py.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes-mb', default='0.25,1,4,16,32,64,132,256')
    ap.add_argument('--dtype', default='float32', choices=['float32', 'bfloat16'])
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    args = ap.parse_args()
    from applestar_amd.parallel import dist as pdist
    rank, world = pdist.init()
    dev = torch.device('cuda', torch.cuda.current_device())
    dtype = getattr(torch, args.dtype)
    avg = dist.get_backend() == 'nccl'
    op = dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM

    def timed(fn):
        ts = []
        for i in range(args.warmup + args.iters):
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            if i >= args.warmup:
                ts.append(time.perf_counter() - t0)
        t = torch.tensor(sorted(ts)[len(ts) // 2], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)

    for mb in [float(x) for x in args.sizes_mb.split(',')]:
        n = int(mb * 2 ** 20 / torch.tensor([], dtype=dtype).element_size())
        buf = torch.ones(n, dtype=dtype, device=dev)
        t = timed(lambda: dist.all_reduce(buf, op=op))
        nbytes = n * buf.element_size()
        if rank == 0:
            print(json.dumps({'kind': 'all_reduce', 'world': world, 'dtype': args.dtype, 'mb': mb,
                              'ms': round(1000 * t, 4), 'busbw_GBps': round(2 * (world - 1) / world * nbytes / t / 1e9, 1),
                              'algbw_GBps': round(nbytes / t / 1e9, 1)}), flush=True)
    # the learner's pattern: flat fp32 master gradient + the fp32-parameter bucket, issued async back to back
    big = torch.ones(33_000_000, dtype=torch.float32, device=dev)
    small = torch.ones(200_000, dtype=torch.float32, device=dev)

    def learner():
        hs = [dist.all_reduce(b, op=op, async_op=True) for b in (big, small)]
        for h in hs:
            h.wait()
        if not avg:
            big.div_(world)
            small.div_(world)
    t = timed(learner)
    if rank == 0:
        print(json.dumps({'kind': 'learner_grad_reduce', 'world': world, 'mb': round((big.numel() + small.numel()) * 4 / 2 ** 20, 1),
                          'ms': round(1000 * t, 4)}), flush=True)
    pdist.finalize()


if __name__ == '__main__':
    main()
