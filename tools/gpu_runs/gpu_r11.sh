#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -k "upsample_conv" -x -q > gpurun_out/r11_upconv.log 2>&1; rc=$?
echo "upconv tests exit $rc"; tail -15 gpurun_out/r11_upconv.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/r11_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r11_bench.log | cut -c1-250
