set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "maxpool or handoff or resblock or spatial or trainer or step" > gpurun_out/pool_pytest.txt 2>&1 || { tail -40 gpurun_out/pool_pytest.txt; exit 1; }
tail -2 gpurun_out/pool_pytest.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/pool_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pool_f32_$i.json'));print('fp32 pooled-mask', $i, d['ms_per_step'])"
  APPLESTAR_POOL_BWD_RELU=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/pool0_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/pool0_f32_$i.json'));print('fp32 full-res mask', $i, d['ms_per_step'])"
done
