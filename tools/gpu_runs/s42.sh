set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_model_parity_gpu.py tests/test_model_gpu.py tests/test_glue_fusions_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/s42_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/s42_pytest.txt; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for v in base padded; do
    case $v in base) E="";; padded) E="APPLESTAR_PACKED_KEYS=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s42_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s42_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
  done
done
for v in base padded; do
  case $v in base) E="";; padded) E="APPLESTAR_PACKED_KEYS=0";; esac
done
