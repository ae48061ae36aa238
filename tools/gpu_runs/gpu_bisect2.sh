#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
run() { timeout -k 10 240 python -u tools/graph_bisect.py $1 > gpurun_out/bisect2_$1_$2.log 2>&1; rc=$?
  echo "stage $1 ($2) exit $rc"; grep "^\[" gpurun_out/bisect2_$1_$2.log | tail -2
  if [ $rc -ne 0 ]; then grep -v '^  File "/usr' gpurun_out/bisect2_$1_$2.log | grep -v "^Extension" | tail -25; exit 1; fi; }
run update gs && run fwd_bwd gs && POOL=1 run fwd_bwd pool && POOL=1 run update pool
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -x --timeout 200 --timeout-method thread -k "graphed_train_step" > gpurun_out/r2d_test.log 2>&1; rc=$?
echo "test exit $rc"; grep -v '^  File "/usr' gpurun_out/r2d_test.log | grep -v "^Extension" | tail -25
