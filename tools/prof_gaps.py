"""GPU idle-time attribution for one learner iteration of a rocprofv3 kernel trace.

    python tools/prof_gaps.py <kernel_trace.csv> [n_gaps]

Iteration = the kernels between the last two optimizer bursts (fused Adam).  Prints the wall time,
the union of kernel-busy intervals over all streams (overlap counted once), the summed kernel time,
the idle time (wall - union), and the largest idle gaps with the kernels on either side: idle time
between kernels is host launch / sync latency that a HIP graph would remove.
"""
import csv
import re
import sys


def short(n):
    n = re.sub(r'\(.*', '', n)
    n = re.sub(r'<.*', '', n)
    n = n.replace('void ', '').replace('at::native::', '').replace('(anonymous namespace)::', '')
    if n.startswith('Cijk'):
        m = re.search(r'MT\d+x\d+x\d+', n)
        n = 'GEMM ' + (m.group(0) if m else '')
    return n[:56]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ngap = int(sys.argv[2]) if len(sys.argv) > 2 else 25
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
    start = ends[-2] + 1 if len(ends) >= 2 else 0
    it = rows[start:ends[-1] + 1]
    iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r) for r in it]
    t0 = iv[0][0]
    t1 = max(e for _, e, _ in iv)
    busy, gaps = 0, []
    cur_s, cur_e, cur_r = iv[0]
    for s, e, r in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e - t0, cur_r, r))
            cur_s, cur_e, cur_r = s, e, r
        elif e > cur_e:
            cur_e, cur_r = e, r
    busy += cur_e - cur_s
    total = sum(e - s for s, e, _ in iv)
    wall = t1 - t0
    print(f'iteration: {len(it)} kernels  wall {wall / 1e6:.2f} ms  busy(union) {busy / 1e6:.2f} ms  '
          f'sum {total / 1e6:.2f} ms  idle {(wall - busy) / 1e6:.2f} ms  gaps>0: {len(gaps)}')
    edges = [0, 2000, 5000, 10000, 50000, float('inf')]      # ns
    parts = []
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = [g[0] for g in gaps if lo <= g[0] < hi]
        parts.append(f'[{lo / 1e3:g},{hi / 1e3:g}) us: {len(sel)} gaps {sum(sel) / 1e6:.2f} ms')
    print('idle gaps by size: ' + '; '.join(parts))
    print(f'largest {ngap} gaps:')
    for g, at, a, b in sorted(gaps, key=lambda x: -x[0])[:ngap]:
        print(f'  {g / 1e3:8.1f} us at {at / 1e6:7.2f} ms  after {short(a["Kernel_Name"]):56s} before {short(b["Kernel_Name"])}')


if __name__ == '__main__':
    main()
