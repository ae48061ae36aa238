set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_flat_model.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r5l_inf_pytest.txt 2>&1; rc=$?
grep -E "PASS|FAIL|^E |passed|failed" gpurun_out/r5l_inf_pytest.txt | tail -30; ok $rc || exit 1
timeout -k 10 200 python -u tools/inference_casts.py --batch 1 --top 50 > gpurun_out/r5l_inference_casts.txt 2>&1 || { tail -20 gpurun_out/r5l_inference_casts.txt; exit 1; }
head -60 gpurun_out/r5l_inference_casts.txt
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 40 > gpurun_out/r5l_bench_inference.jsonl 2>&1 || exit 1
cat gpurun_out/r5l_bench_inference.jsonl
APPLESTAR_INFERENCE_FORMS=0 timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 40 > gpurun_out/r5l_bench_inference_noforms.jsonl 2>&1 || exit 1
cat gpurun_out/r5l_bench_inference_noforms.jsonl
