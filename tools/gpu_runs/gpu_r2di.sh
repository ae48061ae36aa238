#!/bin/bash
# BO encoder: test + kernel stats of the bench step + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "bo_encoder" -x -q --timeout 120 --timeout-method thread > gpurun_out/r2di_bo_tests.log 2>&1 || { tail -40 gpurun_out/r2di_bo_tests.log; exit 1; }
tail -2 gpurun_out/r2di_bo_tests.log
TAG=r2di_prof bash tools/gpu_prof.sh > gpurun_out/r2di_prof_summary.log 2>&1 || { tail -20 gpurun_out/r2di_prof_summary.log; exit 1; }
grep -E "bo_fwd|bo_bwd" gpurun_out/r2di_prof_top.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 4 > gpurun_out/r2di_bench.log 2>&1 || { tail -20 gpurun_out/r2di_bench.log; exit 1; }
tail -1 gpurun_out/r2di_bench.log | cut -c1-200
