#!/bin/bash
# residual-gradient link: new test, full GPU suite, A/B/A/B of APPLESTAR_RESID_LINK, kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_resid_link_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2du_link_test.log 2>&1; rc=$?
grep -E "per-segment|passed|failed" gpurun_out/r2du_link_test.log | tail -3 | cut -c1-600
[ $rc -lt 2 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --deselect tests/test_resid_link_gpu.py::test_grad_link_matches_plain_path_and_fp64 --timeout 120 --timeout-method thread > gpurun_out/r2du_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2du_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r2du_pytest_gpu.log
VAR=APPLESTAR_RESID_LINK bash tools/gpu_ab3.sh | tee gpurun_out/r2du_ab_resid_link.txt || exit 1
TAG=r2du_prof bash tools/gpu_prof.sh > gpurun_out/r2du_prof_summary.log 2>&1 || { tail -20 gpurun_out/r2du_prof_summary.log; exit 1; }
head -12 gpurun_out/r2du_prof_summary.log
