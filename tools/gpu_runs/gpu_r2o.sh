#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "trainer_step or graphed_train" > gpurun_out/r2o.log 2>&1; rc=$?
echo "exit $rc: $(grep -oE 'AssertionError: .*' gpurun_out/r2o.log | head -1 | cut -c1-900) $(tail -1 gpurun_out/r2o.log)"
