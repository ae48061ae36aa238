set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag/poison_probe.py --precision both > gpurun_out/s8_poison_fwd.txt 2>&1 || { tail -30 gpurun_out/s8_poison_fwd.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s8_poison_fwd.txt | head -40
timeout -k 10 300 python -u tools/diag/poison_probe.py --precision both --backward > gpurun_out/s8_poison_bwd.txt 2>&1 || { tail -30 gpurun_out/s8_poison_bwd.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/s8_poison_bwd.txt | head -40
APPLESTAR_LSTM_BF16_OUT=0 timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -x -q -s --timeout 200 --timeout-method thread -k "bf16_gpu_vs_cpu" > gpurun_out/s8_parity_lb0.txt 2>&1; grep -h "selected-units logit error\|passed\|failed" gpurun_out/s8_parity_lb0.txt | tail -3
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_inference_server.py tests/test_model_parity_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread --deselect tests/test_model_parity_gpu.py::test_full_model_bf16_gpu_vs_cpu_fp32 > gpurun_out/s8_pytest.txt 2>&1 || { tail -40 gpurun_out/s8_pytest.txt; exit 1; }
tail -1 gpurun_out/s8_pytest.txt
timeout -k 10 200 python tools/inference_casts.py --batch 1 --top 40 > gpurun_out/s8_inference_casts_b1.txt 2>&1 || exit 1
head -28 gpurun_out/s8_inference_casts_b1.txt
for i in 1 2; do
  for c in 1 0; do
    APPLESTAR_LSTM_BF16_OUT=$c timeout -k 10 300 python tools/bench_inference.py --batches 1,16 --modes policy_graph > gpurun_out/s8_inf_lb${c}_$i.jsonl 2>/dev/null || exit 1
    echo "lstm_bf16_out=$c run $i"; grep -h 'graph' gpurun_out/s8_inf_lb${c}_$i.jsonl | cut -c1-220
  done
done
