set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_inference_server.py tests/test_model_parity_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s7_pytest.txt 2>&1 || { tail -40 gpurun_out/s7_pytest.txt; exit 1; }
tail -1 gpurun_out/s7_pytest.txt
timeout -k 10 200 python tools/inference_casts.py --batch 1 --top 40 > gpurun_out/s7_inference_casts_b1.txt 2>&1 || exit 1
head -30 gpurun_out/s7_inference_casts_b1.txt
for i in 1 2; do
  for c in 1 0; do
    APPLESTAR_LSTM_BF16_OUT=$c timeout -k 10 300 python tools/bench_inference.py --batches 1,16 --modes policy_graph > gpurun_out/s7_inf_lb${c}_$i.jsonl 2>/dev/null || exit 1
    echo "lstm_bf16_out=$c run $i"; grep -h 'graph' gpurun_out/s7_inf_lb${c}_$i.jsonl | cut -c1-220
  done
done
