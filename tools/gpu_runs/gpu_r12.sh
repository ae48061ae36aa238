#!/bin/bash
# Round-1 checkpoint on HEAD: full GPU suite, bench, kernel stats, small-op attribution.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r12_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -3 gpurun_out/r12_pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r12_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r12_bench.log | cut -c1-300
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/elementwise_attrib.py --out gpurun_out/r12_attrib.txt --top 60 > /dev/null 2>&1; rc=$?
echo "attrib exit $rc"; [ $rc -eq 0 ] || exit 1
TAG=r12_prof bash tools/gpu_prof.sh
