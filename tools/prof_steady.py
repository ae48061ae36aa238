"""Steady-state kernel table from a rocprofv3 kernel trace: only the last K learner iterations (iteration =
the kernels between consecutive optimizer bursts), so first-step costs (MIOpen kernel search, lazy
allocations, library heuristics) do not pollute the per-iteration numbers.

    python tools/prof_steady.py <kernel_trace.csv> [K=2] [top=50]
"""
import csv
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from prof_summary import family  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    # optimizer bursts: torch's fused Adam, or the native fused clip + Adam (optim.hip mt_adam_kernel)
    opt = [i for i, r in enumerate(rows) if 'fused_adam' in r['Kernel_Name'].lower() or 'FusedOpti' in r['Kernel_Name']
           or 'mt_adam_kernel' in r['Kernel_Name']]
    ends = []
    for i in opt:
        if not ends or i > ends[-1] + 5:
            ends.append(i)
        else:
            ends[-1] = i
    if len(ends) < K + 1:
        raise SystemExit(f'only {len(ends)} optimizer bursts in the trace')
    sel = rows[ends[-K - 1] + 1:ends[-1] + 1]
    t0 = int(sel[0]['Start_Timestamp'])
    t1 = max(int(r['End_Timestamp']) for r in sel)
    per = defaultdict(lambda: [0.0, 0])
    fam = defaultdict(lambda: [0.0, 0])
    for r in sel:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
        per[r['Kernel_Name']][0] += d
        per[r['Kernel_Name']][1] += 1
        f = family(r['Kernel_Name'])
        fam[f][0] += d
        fam[f][1] += 1
    tot = sum(v[0] for v in per.values()) / K
    print(f'steady state, last {K} iterations: {len(sel) / K:.0f} kernels / iteration, kernel time {tot:.2f} ms / '
          f'iteration, wall {(t1 - t0) / 1e6 / K:.2f} ms / iteration')
    for f, (d, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f'  {d / K:8.2f} ms {100 * d / K / tot:5.1f}%  {n / K:6.0f} launches  {f}')
    print()
    for name, (d, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:top]:
        short = re.sub(r'\s+', ' ', name)[:160]
        print(f'{d / K:8.3f} ms/it {n / K:6.1f} calls/it  {short}')


if __name__ == '__main__':
    main()
