"""Do kernels on two HIP streams run concurrently on this box?  A one-workgroup spin kernel
(torch.cuda._sleep) on stream A and a chain of GEMMs on stream B, timed alone and together; prints one
JSON line (overlap = (tA + tB - t_both) / min(tA, tB): 1 = fully concurrent, 0 = serialised)."""
import json
import time

import torch


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t


def main():
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.randn(4096, 4096, device='cuda', dtype=torch.bfloat16)
    cycles = 20_000_000

    def spin():
        with torch.cuda.stream(a):
            torch.cuda._sleep(cycles)

    def gemms():
        with torch.cuda.stream(b):
            for _ in range(60):
                torch.mm(x, x)

    for _ in range(2):
        spin(), gemms()
    ta = min(timed(spin) for _ in range(3))
    tb = min(timed(gemms) for _ in range(3))
    tab = min(timed(lambda: (spin(), gemms())) for _ in range(3))
    print(json.dumps({'spin_ms': round(1e3 * ta, 3), 'gemms_ms': round(1e3 * tb, 3), 'both_ms': round(1e3 * tab, 3),
                      'overlap': round((ta + tb - tab) / min(ta, tb), 3)}), flush=True)


if __name__ == '__main__':
    main()
