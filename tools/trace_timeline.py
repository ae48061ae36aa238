"""Kernel timeline of the last N dispatches in a rocprofv3 kernel trace: start offset, duration and the idle gap
before each kernel, plus the totals (busy vs gap) of the window - the view of one HIP-graph replay's critical path.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python tools/bench_inference.py ...
    python tools/trace_timeline.py OUT --last 200 [--split-ms 0.2]

``--split-ms``: a gap longer than this starts a new group (a new replay); only the last group is printed.
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out_dir')
    ap.add_argument('--last', type=int, default=400)
    ap.add_argument('--split-ms', type=float, default=0.0, help='0: no grouping, print the whole window')
    args = ap.parse_args()
    files = glob.glob(os.path.join(args.out_dir, '**', '*kernel_trace.csv'), recursive=True)
    if not files:
        raise SystemExit(f'no kernel_trace.csv under {args.out_dir}')
    rows = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    rows = rows[-args.last:]
    # the last group: walk back from the end until a gap longer than split
    i = len(rows) - 1
    if args.split_ms <= 0:
        i = 0
    while i > 0 and rows[i][0] - rows[i - 1][1] <= args.split_ms * 1e6:
        i -= 1
    grp = rows[i:]
    t0 = grp[0][0]
    busy = gap = 0
    prev_end = None
    print(f'{len(grp)} kernels, span {(grp[-1][1] - t0) / 1e3:.1f} us')
    print(f'{"start_us":>9} {"dur_us":>7} {"gap_us":>7}  kernel')
    for s, e, n in grp:
        g = 0 if prev_end is None else max(0, s - prev_end)
        gap += g
        busy += e - s
        print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {g / 1e3:7.1f}  {n[:110]}')
        prev_end = e if prev_end is None else max(prev_end, e)
    print(f'busy {busy / 1e3:.1f} us, gaps {gap / 1e3:.1f} us')


if __name__ == '__main__':
    main()
