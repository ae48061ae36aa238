#!/bin/bash
# Capture bisection: stages in order, stop at the first failure (a crash ends the call).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for st in ${STAGES:-fwd_nograd fwd fwd_loss fwd_bwd_nomaster fwd_bwd update}; do
  timeout -k 10 240 python -u tools/graph_bisect.py $st > gpurun_out/bisect_$st.log 2>&1; rc=$?
  echo "stage $st exit $rc"; grep "^\[" gpurun_out/bisect_$st.log | tail -3
  if [ $rc -ne 0 ]; then grep -v '^  File "/usr' gpurun_out/bisect_$st.log | grep -v "^Extension" | tail -25; exit 1; fi
done
