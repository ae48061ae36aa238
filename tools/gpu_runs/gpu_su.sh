#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -k su_sample -x -q > gpurun_out/su_test.log 2>&1; rc=$?; echo "su test exit $rc"; tail -30 gpurun_out/su_test.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/bench_inference.py > gpurun_out/su_infer.log 2>&1; echo "infer exit $?"; cat gpurun_out/su_infer.log | grep batch
