#!/bin/bash
# end-of-session kernel profile (rocprofv3 kernel trace + stats) of the bench step
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
TAG=r2dz_prof bash tools/gpu_prof.sh > gpurun_out/r2dz_prof_summary.log 2>&1 || { tail -20 gpurun_out/r2dz_prof_summary.log; exit 1; }
head -12 gpurun_out/r2dz_prof_summary.log
