#!/bin/bash
# Session-2 GPU check: new-kernel tests, all gpu tests, bench, rocprofv3 kernel stats of the bench step.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
mkdir -p gpurun_out
TAG=${TAG:-s2}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "${KSEL:-maxpool or segment or conv}" > gpurun_out/${TAG}_new.log 2>&1; rc=$?
echo "new-kernel tests exit $rc"; tail -4 gpurun_out/${TAG}_new.log
[ $rc -eq 0 ] || exit 1
if [ "${MICRO:-1}" = "1" ]; then
  timeout -k 10 300 python -u tools/bench_conv.py > gpurun_out/${TAG}_micro.jsonl 2>&1 || { tail -20 gpurun_out/${TAG}_micro.jsonl; exit 1; }
  cat gpurun_out/${TAG}_micro.jsonl
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -4 gpurun_out/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
if [ "${PROFILE:-1}" = "1" ]; then
  TAG=${TAG}_prof bash tools/gpu_prof.sh || exit 1
fi
