#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
b() { timeout -k 10 300 env "$@" python bench.py --steps 15 --warmup 4 > gpurun_out/ab_$1.log 2>&1; rc=$?; echo "$* exit $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$1.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/ab_$1.log)"; [ $rc -lt 124 ] || exit 1; }
b X=1
b APPLESTAR_AMP_CACHE=1
b APPLESTAR_HEAD_STATS_NATIVE=0
b APPLESTAR_AMP_CACHE=1 APPLESTAR_HEAD_STATS_NATIVE=0
