set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small or wgrad or linear_f32" > gpurun_out/s4_pytest.txt 2>&1 || { tail -40 gpurun_out/s4_pytest.txt; exit 1; }
tail -1 gpurun_out/s4_pytest.txt
for i in 1 2; do
  for w in 16 4; do
    APPLESTAR_SMALL_TN_WAVES=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s4_fp32_w${w}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s4_fp32_w${w}_$i.json'));print('fp32 small_tn waves=$w', $i, d['ms_per_step'])"
  done
done
for i in 1 2; do
  for w in 16 4; do
    APPLESTAR_SMALL_TN_WAVES=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s4_bf16_w${w}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s4_bf16_w${w}_$i.json'));print('bf16 small_tn waves=$w', $i, d['ms_per_step'])"
  done
done
