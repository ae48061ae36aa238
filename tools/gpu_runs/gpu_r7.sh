#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
echo "ring test"
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -k ring -x -q > gpurun_out/r7_ring_test.log 2>&1; rc=$?; echo "ring test exit $rc"; tail -3 gpurun_out/r7_ring_test.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_ring.py > gpurun_out/r7_ring.log 2>&1; echo "ring bench exit $?"; tail -2 gpurun_out/r7_ring.log
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r7_pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r7_pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r7_bench.log 2>&1; echo "bench exit $?"; tail -1 gpurun_out/r7_bench.log | cut -c1-200
