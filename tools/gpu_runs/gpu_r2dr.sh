#!/bin/bash
# joint SU/TU key projection: full GPU suite, A/B/A/B, kernel profile of the resulting state
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2dr_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r2dr_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2dr_pytest_gpu.log
VAR=APPLESTAR_JOINT_KEYS bash tools/gpu_ab3.sh || exit 1
TAG=r2dr_prof bash tools/gpu_prof.sh > gpurun_out/r2dr_prof_summary.log 2>&1 || { tail -20 gpurun_out/r2dr_prof_summary.log; exit 1; }
head -12 gpurun_out/r2dr_prof_summary.log
