set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_model_parity_gpu.py tests/test_model_gpu.py tests/test_phased_backward_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s14_pytest.txt 2>&1 || { tail -40 gpurun_out/s14_pytest.txt; exit 1; }
tail -1 gpurun_out/s14_pytest.txt
for i in 1 2; do
  for v in new old; do
    case $v in new) E="";; old) E="APPLESTAR_KEYS_SIDE=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s14_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s14_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s14_bf16_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s14_bf16_${v}_$i.json'));print('bf16 $v', $i, d['ms_per_step'])"
  done
done
