"""For the kernels matching a pattern in the last learner iteration of a rocprofv3 kernel_trace.csv: their
duration and how much other kernel time ran concurrently inside their interval (clipped), by kernel.  Shows
whether latency-bound kernels (the 8-workgroup LSTM recurrence) share the GPU with independent work.

    python tools/overlap_around.py <kernel_trace.csv> <regex> [top]
"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = re.compile(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 8
rows.sort(key=lambda r: int(r['Start_Timestamp']))
opt = [i for i, r in enumerate(rows) if 'FusedOpti' in r['Kernel_Name'] or 'fused_adam' in r['Kernel_Name'].lower()
       or 'mt_adam_kernel' in r['Kernel_Name']]
ends = []
for i in opt:
    if not ends or i > ends[-1] + 5:
        ends.append(i)
    else:
        ends[-1] = i
it = rows[ends[-2] + 1:ends[-1] + 1] if len(ends) >= 2 else rows
iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in it]


def short(n):
    n = n.replace('(anonymous namespace)::', '')
    n = re.sub(r'\(.*', '', n)
    return n.split('::')[-1][:70]


for s, e, n in iv:
    if not pat.search(n):
        continue
    other = collections.Counter()
    for s2, e2, n2 in iv:
        if (s2, e2, n2) == (s, e, n):
            continue
        ov = min(e, e2) - max(s, s2)
        if ov > 0:
            other[short(n2)] += ov
    tot = sum(other.values())
    print(f'{short(n)}  {(e - s) / 1e3:8.1f} us   concurrent kernel time {tot / 1e3:8.1f} us')
    for k, v in other.most_common(top):
        print(f'      {v / 1e3:8.1f} us  {k}')
