set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "relu_mask_handoff or layer_norm or transformer" -q --timeout 120 --timeout-method thread > gpurun_out/s33_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/s33_pytest.txt; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for v in base nolnm; do
    case $v in base) E="";; nolnm) E="APPLESTAR_LN_RELU_MASK=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s33_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s33_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
  done
done
