set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
APPLESTAR_RUN_SLOW=1 timeout -k 20 900 python -u -m pytest tests/test_learning_pipeline_gpu.py -v -s --timeout 420 --timeout-method thread > gpurun_out/r8c_pytest_learn.txt 2>&1; rc=$?
grep -E '"progress"|PASSED|FAILED|passed|failed' gpurun_out/r8c_pytest_learn.txt | tail -14; exit $rc
