#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "conv3x3 or resblock or gated" > gpurun_out/r2t_k.log 2>&1; rc=$?
echo "targeted exit $rc"; tail -2 gpurun_out/r2t_k.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r2t_k.log | head -20; exit 1; }
timeout -k 10 300 python tools/bench_conv_halo.py > gpurun_out/r2t_conv.jsonl 2>&1; rc=$?; echo "conv bench exit $rc"; cat gpurun_out/r2t_conv.jsonl; [ $rc -eq 0 ] || exit 1
b() { timeout -k 10 300 env "$@" python bench.py --steps 15 --warmup 4 > gpurun_out/r2t_ab_$1.log 2>&1; rc=$?; echo "$* exit $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2t_ab_$1.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/r2t_ab_$1.log)"; [ $rc -lt 124 ] || exit 1; }
b APPLESTAR_CONV_HALO=1
b APPLESTAR_CONV_HALO=0
