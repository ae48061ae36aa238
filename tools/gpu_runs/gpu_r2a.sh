#!/bin/bash
# Round-2 first GPU call: wgrad discriminating run (plain + NaN-poisoned partials), GPU suite, bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] && { echo "fatal exit $1: stopping"; exit 1; }; return 0; }
timeout -k 10 300 python -u tools/wgrad_diag.py --iters 30 --out gpurun_out/r2a_wgrad_diag.jsonl > gpurun_out/r2a_wgrad_diag.log 2>&1; rc=$?
echo "wgrad_diag exit $rc"; tail -2 gpurun_out/r2a_wgrad_diag.log; fatal $rc
APPLESTAR_WGRAD_NANFILL=1 timeout -k 10 300 python -u tools/wgrad_diag.py --iters 30 --out gpurun_out/r2a_wgrad_diag.jsonl > gpurun_out/r2a_wgrad_diag_nan.log 2>&1; rc=$?
echo "wgrad_diag nanfill exit $rc"; tail -1 gpurun_out/r2a_wgrad_diag_nan.log; fatal $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r2a_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -3 gpurun_out/r2a_pytest_gpu.log; fatal $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r2a_bench.log 2>&1; rc=$?
echo "bench exit $rc"; tail -1 gpurun_out/r2a_bench.log | cut -c1-400; fatal $rc
