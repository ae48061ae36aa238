#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
run() { timeout -k 10 240 python -u tools/graph_bisect.py $1 > gpurun_out/bisect3_$1_$2.log 2>&1; rc=$?
  echo "stage $1 ($2) exit $rc"; grep "^\[" gpurun_out/bisect3_$1_$2.log | tail -2
  if [ $rc -ne 0 ]; then grep -v '^  File "/usr' gpurun_out/bisect3_$1_$2.log | grep -v "^Extension" | tail -25; exit 1; fi; }
SIDE=1 run fwd side_in_capture
SIDE_WARM=1 run fwd_bwd sidewarm
