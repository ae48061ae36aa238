"""Host and device cost of staging one RL learner batch to the GPU: per-tensor ``.to(device)`` vs the
packed single-buffer copy (runtime/prefetch.py).  Prints one JSON line per mode."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from applestar_amd.rl.synthetic import rl_batch  # noqa: E402
from applestar_amd.runtime import prefetch as P  # noqa: E402


def main():
    dev = torch.device('cuda', 0)
    host = P.pack_tree(rl_batch(6, 64, seed=0))
    side = torch.cuda.Stream(dev)
    compute = torch.cuda.current_stream(dev)
    for mode in ('per_tensor', 'packed', 'per_tensor', 'packed'):
        host_t, wall_t = 0.0, 0.0
        for i in range(12):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(side):
                out = host.to_device(dev, record_stream=compute) if mode == 'packed' else \
                    P._to_side(dict(host), dev, compute)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if i >= 2:
                host_t += t1 - t0
                wall_t += t2 - t0
            del out
        print(json.dumps({'mode': mode, 'host_ms': round(host_t * 100, 3), 'wall_ms': round(wall_t * 100, 3),
                          'bytes_mb': round(host.buffer.numel() / 1e6, 1)}), flush=True)


if __name__ == '__main__':
    main()
