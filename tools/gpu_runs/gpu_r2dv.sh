#!/bin/bash
# attention backward vs fp32 as the score scale grows
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 200 python -u tools/diag/attn_scale_diag.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r2dv_attn_scale_diag.txt
