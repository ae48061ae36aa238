#!/bin/bash
# rocprofv3 kernel stats of bench.py (kernel-trace only, no counters) -> gpurun_out/<TAG>_{families,top,gaps}.txt
#   TAG=r3b_fp32 ITERS=5 BENCH_ARGS="--precision fp32 --steps 5 --warmup 3 --inference 0" bash tools/gpu_prof.sh
# ITERS = profiled learner iterations the per-iteration numbers are divided by (warm-up + timed steps).
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-prof}
ITERS=${ITERS:-5}
BENCH_ARGS=${BENCH_ARGS:-"--steps 3 --warmup 2"}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P=/tmp/prof_$TAG
# heartbeat: the first fp32 step compiles MIOpen kernels for ~1-2 min without output
( while sleep 45; do date +%T >> $R/gpurun_out/${TAG}.heartbeat; done ) & HB=$!
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- python3 $R/bench.py $BENCH_ARGS > $R/gpurun_out/${TAG}.log 2>&1; rc=$?
kill $HB 2>/dev/null
echo "rocprof exit $rc"; tail -2 $R/gpurun_out/${TAG}.log | cut -c1-200
f=$(find $P -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $R/gpurun_out/${TAG}_kernel_stats.csv
[ -n "$f" ] && python3 $R/tools/prof_summary.py "$f" $ITERS > $R/gpurun_out/${TAG}_families.txt && head -30 $R/gpurun_out/${TAG}_families.txt
[ -n "$f" ] && python3 - "$f" $ITERS > $R/gpurun_out/${TAG}_top.txt <<'PY'
import csv, sys
it = float(sys.argv[2])
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:80]:
    print(f"{float(r['TotalDurationNs'])/1e6/it:8.3f} ms/it {int(r['Calls'])/it:8.1f} calls/it  {r['Name'][:160]}")
PY
[ $rc -eq 0 ] || exit $rc
t=$(find $P -name '*kernel_trace.csv' | head -1)
[ -n "$t" ] && python3 $R/tools/prof_gaps.py "$t" 30 > $R/gpurun_out/${TAG}_gaps.txt && head -8 $R/gpurun_out/${TAG}_gaps.txt
[ -n "$t" ] && python3 $R/tools/prof_steady.py "$t" ${STEADY:-2} 70 > $R/gpurun_out/${TAG}_steady.txt && head -14 $R/gpurun_out/${TAG}_steady.txt
rm -rf $P
exit 0
