set -o pipefail
mkdir -p gpurun_out
APPLESTAR_TU_SIDE_STREAM=1 APPLESTAR_CRITIC_SIDE_STREAM=1 timeout -k 10 600 python -u -m pytest tests/test_model_parity_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fp32 or trainer" > gpurun_out/s10_pytest.txt 2>&1 || { tail -40 gpurun_out/s10_pytest.txt; exit 1; }
tail -1 gpurun_out/s10_pytest.txt
for i in 1 2; do
  for v in base tu critic; do
    case $v in base) E="";; tu) E="APPLESTAR_TU_SIDE_STREAM=1";; critic) E="APPLESTAR_CRITIC_SIDE_STREAM=1";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s10_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s10_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
  done
done
for i in 1 2; do
  for v in base tu; do
    case $v in base) E="";; tu) E="APPLESTAR_TU_SIDE_STREAM=1";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s10_bf16_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s10_bf16_${v}_$i.json'));print('bf16 $v', $i, d['ms_per_step'])"
  done
done
