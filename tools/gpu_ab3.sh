#!/bin/bash
# A/B/A/B bench of an env toggle: VAR=name (values 1 and 0), 4 runs alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
b() { timeout -k 10 300 env $VAR=$1 python bench.py --steps 15 --warmup 4 > gpurun_out/ab3_$VAR$1_$2.log 2>&1; rc=$?; echo "$VAR=$1 run $2 exit $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab3_$VAR$1_$2.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/ab3_$VAR$1_$2.log)"; [ $rc -lt 124 ] || exit 1; }
b 1 a && b 0 a && b 1 b && b 0 b
