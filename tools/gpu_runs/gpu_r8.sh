#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r8_pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r8_pytest_gpu.log
[ $rc -le 1 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r8_bench.log 2>&1; echo "bench exit $?"; tail -1 gpurun_out/r8_bench.log | cut -c1-200
timeout -k 10 600 python tools/op_profile.py --out gpurun_out/r8_op_profile.txt > gpurun_out/r8_op_profile.log 2>&1; echo "op_profile exit $?"; head -40 gpurun_out/r8_op_profile.txt
