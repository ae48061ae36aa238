#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
run() { timeout -k 10 240 python -u tools/graph_bisect.py $1 > gpurun_out/bisect4_$1.log 2>&1; rc=$?
  echo "stage $1 exit $rc"; grep "^\[" gpurun_out/bisect4_$1.log | tail -12
  if [ $rc -ne 0 ]; then grep -v '^  File "/usr' gpurun_out/bisect4_$1.log | grep -v "^Extension" | tail -25; exit 1; fi; }
run trainer_solo && run trainer_pair
