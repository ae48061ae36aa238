#!/bin/bash
# tiled transpose in the derived-weight refresh: tests, kernel stats, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_derived_weights_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2dj_tests.log 2>&1 || { tail -40 gpurun_out/r2dj_tests.log; exit 1; }
tail -2 gpurun_out/r2dj_tests.log
TAG=r2dj_prof bash tools/gpu_prof.sh > gpurun_out/r2dj_prof_summary.log 2>&1 || { tail -20 gpurun_out/r2dj_prof_summary.log; exit 1; }
grep -E "strided_copy|copyBuffer|bfloat16_copy" gpurun_out/r2dj_prof_top.txt | cut -c1-140
timeout -k 10 300 python bench.py --steps 20 --warmup 4 > gpurun_out/r2dj_bench.log 2>&1 || { tail -20 gpurun_out/r2dj_bench.log; exit 1; }
tail -1 gpurun_out/r2dj_bench.log | cut -c1-200
