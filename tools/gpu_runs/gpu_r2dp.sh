#!/bin/bash
# SU teacher mask via scatter-min: full GPU suite + 2 benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2dp_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2dp_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2dp_pytest_gpu.log
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 4 > gpurun_out/r2dp_bench$i.log 2>&1 || { tail -20 gpurun_out/r2dp_bench$i.log; exit 1; }; tail -1 gpurun_out/r2dp_bench$i.log | cut -c1-200; done
