set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "spatial or parity or fp32_gpu or trainer" > gpurun_out/s26_pytest.txt 2>&1 || { tail -40 gpurun_out/s26_pytest.txt; exit 1; }
tail -1 gpurun_out/s26_pytest.txt
for i in 1 2 3; do
  for v in 1 0; do
    APPLESTAR_POOLED_BWD=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s26_fp32_p${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s26_fp32_p${v}_$i.json'));print('fp32 pooled_bwd=$v', $i, d['ms_per_step'])"
  done
done
