#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "resmlp or bo_encoder or trainer_step or graphed_train" > gpurun_out/r2m_$i.log 2>&1; rc=$?
echo "run $i exit $rc: $(grep -oE 'AssertionError: .*' gpurun_out/r2m_$i.log | head -1 | cut -c1-600) $(tail -1 gpurun_out/r2m_$i.log)"; [ $rc -lt 124 ] || exit 1
done
