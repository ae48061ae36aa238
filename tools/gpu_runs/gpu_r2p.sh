#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
b() { timeout -k 10 300 python bench.py --steps 15 --warmup 4 "$@" > gpurun_out/r2p_$2_$4.log 2>&1; rc=$?; echo "$* exit $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r2p_$2_$4.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/r2p_$2_$4.log)"; [ $rc -lt 124 ] || exit 1; }
b --batch 1 --unroll 2 --max-entities 16
b --batch 1 --unroll 8 --max-entities 64
b --batch 6 --unroll 64 --max-entities 512
