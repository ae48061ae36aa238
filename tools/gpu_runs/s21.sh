set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_model_gpu.py tests/test_inference_server.py tests/test_model_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s21_pytest.txt 2>&1 || { tail -40 gpurun_out/s21_pytest.txt; exit 1; }
tail -1 gpurun_out/s21_pytest.txt
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_inference.py --batches 1,16 --modes policy_graph > gpurun_out/s21_inf_$i.jsonl 2>/dev/null || exit 1
  grep -h 'graph' gpurun_out/s21_inf_$i.jsonl | cut -c1-120
done
