"""One line per kernel of the last learner iteration of a rocprofv3 kernel_trace.csv: start offset (ms),
duration (us), stream id, short name.  For reading the step's schedule (which stream runs what, when).

    python tools/trace_listing.py <kernel_trace.csv> > listing.txt
"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
opt = [i for i, r in enumerate(rows) if 'mt_adam_kernel' in r['Kernel_Name'] or 'FusedOpti' in r['Kernel_Name']]
ends = []
for i in opt:
    if not ends or i > ends[-1] + 5:
        ends.append(i)
    else:
        ends[-1] = i
it = rows[ends[-2] + 1:ends[-1] + 1] if len(ends) >= 2 else rows
t0 = int(it[0]['Start_Timestamp'])


def short(n):
    n = n.replace('void ', '').replace('(anonymous namespace)::', '').replace('at::native::', '')
    n = re.sub(r'\(.*', '', n)
    if n.startswith('Cijk'):
        m = re.search(r'MT\d+x\d+x\d+', n)
        n = 'hipBLASLt ' + (m.group(0) if m else '')
    return n[:90]


for r in it:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e6:8.3f} {(e - s) / 1e3:8.1f} s{r['Stream_Id']} {short(r['Kernel_Name'])}")
