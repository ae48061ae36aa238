#!/bin/bash
# derived-weight forms: new GPU tests, full GPU suite, A/B/A/B of the cache.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
T=r2dc
timeout -k 10 300 python -u -m pytest tests/test_derived_weights_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_derived_tests.log 2>&1 || { tail -40 gpurun_out/${T}_derived_tests.log; exit 1; }
tail -3 gpurun_out/${T}_derived_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.log
VAR=APPLESTAR_DERIVED_WEIGHTS bash tools/gpu_ab3.sh
