#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "resmlp or bo_encoder or trainer_step or graphed_train" > gpurun_out/r2k_k.log 2>&1; rc=$?
echo "targeted exit $rc"; tail -3 gpurun_out/r2k_k.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r2k_k.log | head -20; exit 1; }
b() { timeout -k 10 300 env "$@" python bench.py --steps 15 --warmup 4 > gpurun_out/r2k_ab_$1.log 2>&1; rc=$?; echo "$* exit $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2k_ab_$1.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/r2k_ab_$1.log)"; [ $rc -lt 124 ] || exit 1; }
b APPLESTAR_FUSED_RESMLP=1
b APPLESTAR_FUSED_RESMLP=0
b APPLESTAR_FUSED_RESMLP=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2k_pytest_gpu.log 2>&1; rc=$?
echo "pytest exit $rc"; tail -3 gpurun_out/r2k_pytest_gpu.log
