#!/bin/bash
# GPU validation: new kernels first (short), then the full GPU suite, bench and phase timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -k "lstm or upsample_conv" -x -q > gpurun_out/r10_new_kernels.log 2>&1; rc=$?
echo "new-kernel tests exit $rc"; tail -3 gpurun_out/r10_new_kernels.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/r10_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -4 gpurun_out/r10_pytest_gpu.log; fatal $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r10_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r10_bench.log | cut -c1-300; fatal $rc
timeout -k 10 600 python tools/phase_timing.py > gpurun_out/r10_phases.log 2>&1; rc=$?
echo "phases exit $rc"; tail -16 gpurun_out/r10_phases.log
