#!/bin/bash
# One PMC pass (kernel-trace only, <= 8 SQ counters) over a microbenchmark; per-kernel averages.
#   TAG=name FILTER=substr [COUNTERS="..."] bash tools/gpu_pmc.sh python3 tools/bench_x.py child
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-pmc}
COUNTERS=${COUNTERS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS"}
prog=$1; shift
case "$prog" in /*) ;; *) prog=$(command -v $prog) ;; esac
args=()
for a in "$@"; do case "$a" in tools/*) args+=("$R/$a") ;; *) args+=("$a") ;; esac; done
timeout -s KILL 120 rocprofv3 --pmc $COUNTERS -d $R/gpurun_out/$TAG -o run --output-format csv -- "$prog" "${args[@]}" > $R/gpurun_out/$TAG.log 2>&1; rc=$?
echo "pmc exit $rc"; tail -3 $R/gpurun_out/$TAG.log
f=$(find $R/gpurun_out/$TAG -name '*counter_collection.csv' | head -1)
[ -n "$f" ] && FILTER="$FILTER" python3 - "$f" <<'PY' | tee $R/gpurun_out/${TAG}_summary.txt
import csv, sys, collections, os
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
flt = os.environ.get('FILTER', '')
for r in rows:
    k = r['Kernel_Name'][:70]
    if flt not in k:
        continue
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    n = max(max(cnt[(k, c)] for c in d), 1)
    print(k, {c: round(v / n) for c, v in sorted(d.items())})
PY
exit $rc
