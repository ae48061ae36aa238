#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -k lstm -x -q > gpurun_out/r9_lstm_test.log 2>&1; rc=$?; echo "lstm tests exit $rc"; tail -3 gpurun_out/r9_lstm_test.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r9_pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/r9_pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r9_bench.log 2>&1; echo "bench exit $?"; tail -1 gpurun_out/r9_bench.log | cut -c1-200
timeout -k 10 600 python tools/phase_timing.py > gpurun_out/r9_phases.log 2>&1; echo "phases exit $?"; tail -16 gpurun_out/r9_phases.log
