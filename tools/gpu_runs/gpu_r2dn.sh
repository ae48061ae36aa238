#!/bin/bash
# where the forward copies / casts come from (aten op + innermost applestar_amd frame)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python tools/cast_sources.py > gpurun_out/r2dn_cast_sources.txt 2>&1 || { tail -20 gpurun_out/r2dn_cast_sources.txt; exit 1; }
head -70 gpurun_out/r2dn_cast_sources.txt
