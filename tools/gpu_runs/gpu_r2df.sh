#!/bin/bash
# value encoder after the core LSTM: model GPU tests, A/B/A/B, then a trace of what overlaps the LSTM.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_derived_weights_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2df_model_tests.log 2>&1 || { tail -40 gpurun_out/r2df_model_tests.log; exit 1; }
tail -2 gpurun_out/r2df_model_tests.log
VAR=APPLESTAR_VE_AFTER_CORE bash tools/gpu_ab3.sh || exit 1
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $R/gpurun_out/r2df_prof -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/r2df_prof.log 2>&1 || exit 1
t=$(find $R/gpurun_out/r2df_prof -name '*kernel_trace.csv' | head -1)
python3 $R/tools/overlap_around.py "$t" 'lnlstm|bo_bwd|bo_fwd' 6 > $R/gpurun_out/r2df_overlap.txt
python3 $R/tools/prof_gaps.py "$t" 10 > $R/gpurun_out/r2df_gaps.txt
rm -f "$t"
head -50 $R/gpurun_out/r2df_overlap.txt
