"""Per-process summary of a rocprofv3 kernel + memory-copy trace of the single-GPU pipeline
(tools/bench_pipeline.py): for every traced process the kernel count, the union of its kernel intervals (busy
time), the top kernels, and - for the learner (the process that runs the optimizer kernel) - the per-step span,
busy time and idle gaps between consecutive optimizer launches; copies per process (count, bytes, time).

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run_%pid% -- \
        python tools/bench_pipeline.py --envs 8 ...
    python tools/pipeline_trace_summary.py OUT
"""
import argparse
import collections
import csv
import glob
import os
import re


def _union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('out_dir')
    ap.add_argument('--step-kernel', default='mt_adam_kernel')
    args = ap.parse_args()
    kfiles = glob.glob(os.path.join(args.out_dir, '**', '*kernel_trace.csv'), recursive=True)
    cfiles = glob.glob(os.path.join(args.out_dir, '**', '*memory_copy_trace.csv'), recursive=True)
    procs = collections.defaultdict(list)
    for fn in kfiles:
        pid = re.search(r'run_(\d+)', fn)
        key = pid.group(1) if pid else fn
        with open(fn) as f:
            for r in csv.DictReader(f):
                procs[key].append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    copies = collections.defaultdict(list)
    for fn in cfiles:
        pid = re.search(r'run_(\d+)', fn)
        key = pid.group(1) if pid else fn
        with open(fn) as f:
            for r in csv.DictReader(f):
                copies[key].append((int(r['Start_Timestamp']), int(r['End_Timestamp']), int(r.get('Bytes', 0) or 0),
                                    r.get('Direction', r.get('Kind', ''))))
    t_all = [s for v in procs.values() for s, _, _ in v]
    t0 = min(t_all) if t_all else 0
    for key, ks in sorted(procs.items(), key=lambda kv: -len(kv[1])):
        ks.sort()
        span = (ks[-1][1] - ks[0][0]) / 1e6
        busy = _union([(s, e) for s, e, _ in ks]) / 1e6
        print(f'process {key}: {len(ks)} kernels over {span:.1f} ms, busy {busy:.1f} ms '
              f'({100 * busy / max(span, 1e-9):.0f} %), first at {(ks[0][0] - t0) / 1e9:.1f} s')
        top = collections.Counter()
        for s, e, n in ks:
            top[n[:90]] += e - s
        for n, d in top.most_common(6):
            print(f'    {d / 1e6:9.1f} ms  {n}')
        steps = [s for s, e, n in ks if args.step_kernel in n]
        if len(steps) >= 3:
            # per learner step: window between consecutive optimizer launches (skip the first two)
            rows = []
            for a, b in zip(steps[2:-1], steps[3:]):
                w = [(s, e) for s, e, _ in ks if a <= s < b]
                rows.append(((b - a) / 1e6, _union(w) / 1e6, len(w)))
            if rows:
                n = len(rows)
                print(f'    learner steps: {n}, mean span {sum(r[0] for r in rows) / n:.1f} ms, mean kernel busy '
                      f'{sum(r[1] for r in rows) / n:.1f} ms, mean kernels {sum(r[2] for r in rows) / n:.0f}')
                for r in rows[:8]:
                    print(f'      span {r[0]:7.1f} ms  busy {r[1]:6.1f} ms  kernels {r[2]}')
                # the learner's gaps: largest idle intervals inside its steps
                gaps = []
                ks_in = [(s, e, nm) for s, e, nm in ks if steps[2] <= s < steps[-1]]
                for (s0, e0, n0), (s1, e1, n1) in zip(ks_in, ks_in[1:]):
                    if s1 - e0 > 2e6:
                        gaps.append(((s1 - e0) / 1e6, n0[:50], n1[:50]))
                gaps.sort(reverse=True)
                print(f'    idle gaps > 2 ms inside learner steps: {len(gaps)}, total {sum(g[0] for g in gaps):.1f} ms')
                for g in gaps[:12]:
                    print(f'      {g[0]:7.1f} ms  after {g[1]}  before {g[2]}')
        cs = copies.get(key, [])
        if cs:
            by = collections.defaultdict(lambda: [0, 0, 0])
            for s, e, nb, d in cs:
                by[d][0] += 1
                by[d][1] += nb
                by[d][2] += e - s
            for d, (c, nb, dt) in by.items():
                print(f'    copies {d}: {c}, {nb / 1e6:.1f} MB, {dt / 1e6:.1f} ms')


if __name__ == '__main__':
    main()
