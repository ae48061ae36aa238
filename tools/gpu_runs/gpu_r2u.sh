#!/bin/bash
# PMC pass on the conv microbenchmark (halo kernel): stall / MFMA / LDS counters, kernel-trace only.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
export APPLESTAR_CONV_HALO=${HALO:-1}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $R/gpurun_out/r2u_pmc_h$APPLESTAR_CONV_HALO -o run --output-format csv -- python3 $R/tools/bench_conv_halo.py child > $R/gpurun_out/r2u_pmc_h$APPLESTAR_CONV_HALO.log 2>&1; rc=$?
echo "pmc exit $rc"; tail -3 $R/gpurun_out/r2u_pmc_h$APPLESTAR_CONV_HALO.log
f=$(find $R/gpurun_out/r2u_pmc_h$APPLESTAR_CONV_HALO -name '*counter_collection.csv' | head -1)
[ -n "$f" ] && python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r['Kernel_Name'][:60]
    agg[k][r['Counter_Name']] += float(r['Counter_Value'])
    cnt[(k, r['Counter_Name'])] += 1
for k, d in agg.items():
    if 'conv3x3' not in k:
        continue
    n = max(cnt[(k, 'SQ_WAVE_CYCLES')], 1)
    print(k, {c: round(v / n) for c, v in sorted(d.items())})
PY
exit $rc
