#!/bin/bash
# bf16-output wgrad: kernel tests, model GPU tests, in-process A/B, bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r13_pytest.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -3 gpurun_out/r13_pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/ab_bench.py --variant wgrad_bf16 --rounds 6 --steps 10 > gpurun_out/r13_ab.log 2>&1; rc=$?
echo "ab exit $rc"; tail -1 gpurun_out/r13_ab.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r13_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r13_bench.log | cut -c1-300
