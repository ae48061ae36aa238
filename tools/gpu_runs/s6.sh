set -o pipefail
mkdir -p gpurun_out
APPLESTAR_DEFER_STREAMS=3 timeout -k 10 400 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_phased_backward_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "defer or phased" > gpurun_out/s6_pytest.txt 2>&1 || { tail -40 gpurun_out/s6_pytest.txt; exit 1; }
tail -1 gpurun_out/s6_pytest.txt
for i in 1 2; do
  for n in 3 1 2; do
    APPLESTAR_DEFER_STREAMS=$n timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s6_fp32_ds${n}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s6_fp32_ds${n}_$i.json'));print('fp32 defer_streams=$n', $i, d['ms_per_step'])"
  done
done
