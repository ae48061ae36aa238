"""The persistent selected-units sampler (csrc/kernels/pointer.hip) alone: time per launch at B = 1 / 16 over
1, 16 and 64 pointer steps (the slope is the per-step cost, the intercept the prologue), both kernel variants
(APPLESTAR_SU_WIDE), and whether the variants pick the same units.

    python tools/bench_su_sample.py [iters]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    from applestar_amd.ops import native
    from applestar_amd.models.heads import SelectedUnitsHead
    native.ensure_loaded()
    dev = torch.device('cuda', 0)
    torch.manual_seed(3)
    head = SelectedUnitsHead(extra_units=True).to(dev).eval()
    captured = {}
    real = native.su_sample

    def grab(*a):
        captured['args'] = a
        return real(*a)
    native.su_sample = grab
    N = 300
    with torch.no_grad():
        for B in (1, 16):
            ae0 = torch.randn(B, 1024, device=dev)
            ent = torch.randn(B, N, 256, device=dev)
            en = torch.full((B,), N, device=dev)
            su_mask = torch.ones(B, dtype=torch.bool, device=dev)
            u = torch.rand(B, 64, device=dev) * 0.999      # keeps the end token (the last entry) unlikely
            head.forward_sample(ae0, ent, en, su_mask, 1.0, u=u)
            a = list(captured['args'])
            picks = {}
            for v in ('1', '0'):
                os.environ["APPLESTAR_SU_WIDE"] = v
                for steps in (1, 16, 64):
                    a2 = list(a)
                    a2[2] = a[2][:, :steps].contiguous()
                    a2[13] = steps
                    out = real(*a2)
                    for _ in range(3):
                        real(*a2)
                    torch.cuda.synchronize()
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                    ts = []
                    for _ in range(iters):
                        ev[0].record()
                        real(*a2)
                        ev[1].record()
                        torch.cuda.synchronize()
                        ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
                    ts.sort()
                    if steps == 64:
                        picks[v] = (out[1].clone(), out[3].clone())
                    print(json.dumps({'B': B, "wide": v == "1", 'steps': steps, 'us_med': round(ts[len(ts) // 2], 1),
                                      'us_min': round(ts[0], 1), 'su_num_mean': float(out[3].float().mean())}),
                          flush=True)
            same = sum(int(torch.equal(picks['1'][0][b, :int(picks['1'][1][b])],
                                       picks['0'][0][b, :int(picks['0'][1][b])])) for b in range(B))
            print(json.dumps({'B': B, 'rows_same_picks_wide_vs_256': same, 'rows': B}), flush=True)
    os.environ.pop('APPLESTAR_SU_WIDE', None)


if __name__ == '__main__':
    main()
