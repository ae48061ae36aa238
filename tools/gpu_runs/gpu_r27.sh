#!/bin/bash
# conv_wt kernel: its test + conv/resblock tests, full GPU suite, then the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "conv_wt or resblock or conv3x3" -x -q --timeout 120 --timeout-method thread > gpurun_out/r27_new.log 2>&1; rc=$?
echo "new tests exit $rc"; tail -3 gpurun_out/r27_new.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r27_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -3 gpurun_out/r27_pytest_gpu.log; fatal $rc
for i in 1 2; do
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r27_bench$i.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r27_bench$i.log | cut -c1-330; fatal $rc
done
