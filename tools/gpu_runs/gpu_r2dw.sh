#!/bin/bash
# transformer-layer gradient vs float64 (native / torch bf16 / fp32), then A/B/A/B of the residual-gradient link
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 200 python -u tools/diag/layer_grad_diag.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r2dw_layer_grad_diag.txt || exit 1
VAR=APPLESTAR_RESID_LINK bash tools/gpu_ab3.sh | tee gpurun_out/r2dw_ab_resid_link.txt || exit 1
VAR=APPLESTAR_RESID_LINK bash tools/gpu_ab3.sh | tee -a gpurun_out/r2dw_ab_resid_link.txt || exit 1
