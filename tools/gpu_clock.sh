#!/bin/bash
# Effective GPU clock and MFMA issue rate per kernel: one rocprofv3 pass with --kernel-trace (durations) and
# GRBM_GUI_ACTIVE / GRBM_COUNT / SQ_INSTS_MFMA / SQ_BUSY_CYCLES counters, joined per dispatch.
#   TAG=name FILTER=substr bash tools/gpu_clock.sh ./tools/mfma_peak
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-clock}
prog=$1; shift
case "$prog" in /*) ;; ./*) prog=$R/${prog#./} ;; *) prog=$(command -v $prog) ;; esac
args=()
for a in "$@"; do case "$a" in tools/*) args+=("$R/$a") ;; *) args+=("$a") ;; esac; done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_MFMA SQ_BUSY_CYCLES \
  -d $R/gpurun_out/$TAG -o run --output-format csv -- "$prog" "${args[@]}" > $R/gpurun_out/$TAG.log 2>&1; rc=$?
echo "clock pass exit $rc"; tail -2 $R/gpurun_out/$TAG.log
c=$(find $R/gpurun_out/$TAG -name '*counter_collection.csv' | head -1)
k=$(find $R/gpurun_out/$TAG -name '*kernel_trace.csv' | head -1)
[ -n "$c" ] && [ -n "$k" ] && FILTER="$FILTER" python3 - "$c" "$k" <<'PY' | tee $R/gpurun_out/${TAG}_summary.txt
import csv, sys, collections, os
flt = os.environ.get('FILTER', '')
cnt = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(sys.argv[1])):
    d = r.get('Dispatch_Id') or r.get('Correlation_Id')
    cnt[d][r['Counter_Name']] = cnt[d].get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
    names[d] = r['Kernel_Name']
dur = {}
for r in csv.DictReader(open(sys.argv[2])):
    d = r.get('Dispatch_Id') or r.get('Correlation_Id')
    dur[d] = (float(r['End_Timestamp']) - float(r['Start_Timestamp'])) * 1e-9
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d, cs in cnt.items():
    n = names[d][:60]
    if flt not in n or d not in dur or dur[d] <= 0:
        continue
    a = agg[n]
    a['n'] += 1
    a['s'] += dur[d]
    for key, v in cs.items():
        a[key] += v
for n, a in agg.items():
    s = a['s']
    print(f"{n:60s} n={int(a['n'])} avg_us={1e6 * s / a['n']:.1f} GRBM_GUI_ACTIVE/s={a['GRBM_GUI_ACTIVE'] / s / 1e9:.3f}G "
          f"GRBM_COUNT/s={a['GRBM_COUNT'] / s / 1e9:.3f}G SQ_BUSY/s={a['SQ_BUSY_CYCLES'] / s / 1e9:.3f}G "
          f"MFMA_inst/s={a['SQ_INSTS_MFMA'] / s / 1e9:.3f}G")
PY
exit $rc
