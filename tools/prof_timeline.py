"""Print the kernel sequence of the last learner iteration in a rocprofv3 kernel_trace.csv,
collapsing consecutive launches of the same short name, to attribute time to model phases."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
opt_idx = [i for i, r in enumerate(rows) if 'FusedOpti' in r['Kernel_Name'] or 'fused_adam' in r['Kernel_Name'].lower()
           or 'mt_adam_kernel' in r['Kernel_Name']]
# iteration = kernels after the second-to-last optimizer burst up to the last one
ends = []
for i in opt_idx:
    if not ends or i > ends[-1] + 5:
        ends.append(i)
    else:
        ends[-1] = i
start = ends[-2] + 1 if len(ends) >= 2 else 0
stop = ends[-1] + 1
it = rows[start:stop]
t0 = int(it[0]['Start_Timestamp'])
wall = (int(it[-1]['End_Timestamp']) - t0) / 1e6
busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in it) / 1e6
print(f'iteration kernels={len(it)} wall={wall:.2f} ms busy={busy:.2f} ms')


def short(n):
    n = re.sub(r'\(.*', '', n)
    n = re.sub(r'<.*', '', n)
    n = n.replace('void ', '').replace('at::native::', '').replace('(anonymous namespace)::', '')
    if n.startswith('Cijk'):
        n = 'GEMM ' + re.search(r'MT\d+x\d+x\d+', n).group(0)
    return n[:60]


thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
acc_name, acc_t, acc_n, acc_start = None, 0.0, 0, 0.0
for r in it:
    n = short(r['Kernel_Name'])
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    if n == acc_name:
        acc_t += d
        acc_n += 1
        continue
    if acc_name and acc_t >= thr:
        print(f'{acc_start:8.2f} ms  {acc_t:7.3f} ms x{acc_n:<4d} {acc_name}')
    acc_name, acc_t, acc_n = n, d, 1
    acc_start = (int(r['Start_Timestamp']) - t0) / 1e6
if acc_name and acc_t >= thr:
    print(f'{acc_start:8.2f} ms  {acc_t:7.3f} ms x{acc_n:<4d} {acc_name}')
