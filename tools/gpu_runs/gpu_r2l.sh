#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
t() { timeout -k 10 300 env "$@" python -u -m pytest tests/test_model_gpu.py -q -x --timeout 200 --timeout-method thread -k graphed_train > gpurun_out/r2l_$1.log 2>&1; rc=$?; echo "$* exit $rc: $(grep -oE 'AssertionError: .*' gpurun_out/r2l_$1.log | head -1) $(tail -1 gpurun_out/r2l_$1.log)"; [ $rc -lt 124 ] || exit 1; }
t APPLESTAR_FUSED_RESMLP=1
t APPLESTAR_FUSED_RESMLP=0
t APPLESTAR_FUSED_RESMLP=1 APPLESTAR_FUSED_BO=0
t APPLESTAR_FUSED_RESMLP=0 APPLESTAR_FUSED_BO=0
