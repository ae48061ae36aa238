#!/bin/bash
# Iteration check on one MI355X: targeted tests (K=pytest -k expr), full GPU suite (FULL=1), bench,
# optional rocprofv3 kernel summary + idle gaps (PROF=1).  TAG names the outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
TAG=${TAG:-iter}
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
if [ -n "$K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "$K" > gpurun_out/${TAG}_k.log 2>&1; rc=$?
  echo "targeted tests exit $rc"; tail -4 gpurun_out/${TAG}_k.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/${TAG}_k.log | head -20; exit 1; }
fi
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log; fatal $rc
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/${TAG}_bench.log | grep -o '"ms_per_step": [0-9.]*'; grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/${TAG}_bench.log; fatal $rc
if [ "${PROF:-0}" = "1" ]; then
  TAG=${TAG}_prof bash tools/gpu_prof.sh
fi
