#!/bin/bash
# rocprofv3 kernel stats of the bench step (kernel-trace only, no counters).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG} -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/${TAG}.log 2>&1; rc=$?
echo "rocprof exit $rc"; tail -2 $R/gpurun_out/${TAG}.log | cut -c1-200
f=$(find $R/gpurun_out/${TAG} -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 $R/tools/prof_summary.py "$f" 5 > $R/gpurun_out/${TAG}_families.txt && head -30 $R/gpurun_out/${TAG}_families.txt
[ -n "$f" ] && python3 - "$f" > $R/gpurun_out/${TAG}_top.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:60]:
    print(f"{float(r['TotalDurationNs'])/5e6:8.3f} ms/it {int(r['Calls'])//5:6d} calls/it  {r['Name'][:150]}")
PY
[ $rc -eq 0 ] || exit $rc
t=$(find $R/gpurun_out/${TAG} -name '*kernel_trace.csv' | head -1)
[ -n "$t" ] && python3 $R/tools/prof_gaps.py "$t" 30 > $R/gpurun_out/${TAG}_gaps.txt && head -8 $R/gpurun_out/${TAG}_gaps.txt
# the raw trace is large: keep only the summaries
[ -n "$t" ] && rm -f "$t"
exit 0
