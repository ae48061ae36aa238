set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
APPLESTAR_RUN_SLOW=1 timeout -k 20 500 python -u -m pytest tests/test_learning_pipeline_gpu.py -v -s --timeout 420 --timeout-method thread -k bf16 > gpurun_out/r8n_pytest_learn_bf16.txt 2>&1; rc=$?
grep -E '"progress"|PASSED|FAILED|passed|failed' gpurun_out/r8n_pytest_learn_bf16.txt | tail -8; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r8n_bench_default.json 2> gpurun_out/r8n_bench_default.log || { tail -5 gpurun_out/r8n_bench_default.log; exit 1; }
cut -c1-1500 gpurun_out/r8n_bench_default.json
