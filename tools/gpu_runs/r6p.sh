set -o pipefail
mkdir -p gpurun_out
for cfg in "A=1" "APPLESTAR_CONV_SMALLM=0" "APPLESTAR_SCALAR_BF16_INFERENCE=0" "APPLESTAR_CONV_SMALLM=0 APPLESTAR_SCALAR_BF16_INFERENCE=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -q -s --timeout 250 --timeout-method thread -k "test_full_model_bf16_gpu_vs_cpu_fp32" > /tmp/r6p.txt 2>&1; rc=$?
  echo "$cfg rc=$rc $(grep 'selected-units logit error' /tmp/r6p.txt)"
done
