#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
t() { timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "$2" > gpurun_out/r2n_$1.log 2>&1; rc=$?; echo "$1 [$2] exit $rc: $(grep -oE 'AssertionError: .*' gpurun_out/r2n_$1.log | head -1 | cut -c1-200) $(tail -1 gpurun_out/r2n_$1.log)"; [ $rc -lt 124 ] || exit 1; }
t a "resmlp or graphed_train"
t b "bo_encoder or graphed_train"
t c "trainer_step or direct_master or graphed_train"
t d "resmlp or trainer_step or graphed_train"
