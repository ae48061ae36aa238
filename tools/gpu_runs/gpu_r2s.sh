#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "wgrad or bo_encoder or resmlp or linear" > gpurun_out/r2s_k.log 2>&1; rc=$?
echo "targeted exit $rc"; tail -2 gpurun_out/r2s_k.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r2s_k.log | head -20; exit 1; }
timeout -k 10 300 python bench.py --steps 15 --warmup 4 > gpurun_out/r2s_bench.log 2>&1; rc=$?
echo "bench exit $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2s_bench.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/r2s_bench.log)"; [ $rc -lt 124 ] || exit 1
timeout -k 10 300 python tools/kernel_sources.py --pattern copyBuffer --pattern 'elementwise|copy_kernel|CatArray|Fill' --out gpurun_out/r2s_ksrc.txt > gpurun_out/r2s_ksrc.log 2>&1; rc=$?
echo "ksrc exit $rc"; head -60 gpurun_out/r2s_ksrc.txt | cut -c1-260
