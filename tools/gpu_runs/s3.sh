set -o pipefail
mkdir -p gpurun_out
APPLESTAR_WGRAD_SMALL_R=96 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad or linear_f32" > gpurun_out/s3_pytest_wgrad.txt 2>&1 || { tail -40 gpurun_out/s3_pytest_wgrad.txt; exit 1; }
tail -1 gpurun_out/s3_pytest_wgrad.txt
for i in 1 2; do
  for r in 96 0 48 192; do
    APPLESTAR_WGRAD_SMALL_R=$r timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s3_fp32_sr${r}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s3_fp32_sr${r}_$i.json'));print('fp32 small_r=$r', $i, d['ms_per_step'])"
  done
done
for i in 1 2; do
  for r in 96 0; do
    APPLESTAR_WGRAD_SMALL_R=$r timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s3_bf16_sr${r}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s3_bf16_sr${r}_$i.json'));print('bf16 small_r=$r', $i, d['ms_per_step'])"
  done
done
