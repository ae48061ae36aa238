set -o pipefail
mkdir -p gpurun_out
for cfg in "APPLESTAR_SMALL_SIGMOID=0" "APPLESTAR_SMALL_ODD=0" "APPLESTAR_SPLITK_NATIVE=0"; do
  echo "== $cfg" >> gpurun_out/z2_bisect.txt
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -q -s --timeout 200 --timeout-method thread -k "test_full_model_bf16_gpu_vs_cpu_fp32" 2>&1 | grep -E "logit errors|passed|failed" >> gpurun_out/z2_bisect.txt
done
exit 0
