#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r6_pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc" | tee -a gpurun_out/r6_pytest_gpu.log; tail -3 gpurun_out/r6_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python tools/bench_ring.py > gpurun_out/r6_ring.log 2>&1; echo "ring exit $?"; tail -2 gpurun_out/r6_ring.log
timeout -k 10 600 python bench.py --steps 10 --warmup 5 > gpurun_out/r6_bench.log 2>&1; echo "bench exit $?"; tail -1 gpurun_out/r6_bench.log | cut -c1-220
