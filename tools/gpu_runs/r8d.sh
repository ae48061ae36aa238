set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_conv_psb.py 30 psb v0 v1 v2 v3 psb v0 > gpurun_out/r8d_conv_v2.jsonl 2>&1 || { tail -20 gpurun_out/r8d_conv_v2.jsonl; exit 1; }
cat gpurun_out/r8d_conv_v2.jsonl
timeout -k 10 400 python -u -m pytest tests/test_phased_backward_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r8d_pytest_phased.txt 2>&1; rc=$?
tail -4 gpurun_out/r8d_pytest_phased.txt; [ $rc -eq 0 ] || exit 1
APPLESTAR_RUN_SLOW=1 timeout -k 20 500 python -u -m pytest tests/test_learning_pipeline_gpu.py -v -s --timeout 420 --timeout-method thread -k bf16 > gpurun_out/r8d_pytest_learn_bf16.txt 2>&1; rc=$?
grep -E '"progress"|PASSED|FAILED|passed|failed' gpurun_out/r8d_pytest_learn_bf16.txt | tail -8; exit $rc
