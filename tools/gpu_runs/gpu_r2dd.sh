#!/bin/bash
# kernel trace of the bench step: what runs concurrently with the LSTM recurrences and the BO encoder.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2dd_prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r2dd_prof.log 2>&1; rc=$?
echo "rocprof exit $rc"
[ $rc -eq 0 ] || exit $rc
t=$(find $R/gpurun_out/r2dd_prof -name '*kernel_trace.csv' | head -1)
f=$(find $R/gpurun_out/r2dd_prof -name '*kernel_stats.csv' | head -1)
python3 $R/tools/overlap_around.py "$t" 'lnlstm|bo_bwd|bo_fwd|attn_bwd' 6 > $R/gpurun_out/r2dd_overlap.txt
python3 $R/tools/prof_gaps.py "$t" 30 > $R/gpurun_out/r2dd_gaps.txt
python3 $R/tools/prof_summary.py "$f" 5 > $R/gpurun_out/r2dd_families.txt
head -60 $R/gpurun_out/r2dd_overlap.txt
rm -f "$t"
