set -o pipefail
mkdir -p gpurun_out
APPLESTAR_CONV_V2_NARROW_SUB=2 timeout -k 10 400 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "v2_variants or conv3x3_f32" > gpurun_out/s19_pytest.txt 2>&1 || { tail -40 gpurun_out/s19_pytest.txt; exit 1; }
tail -1 gpurun_out/s19_pytest.txt
export CONV_SHAPES="384,38,40,128,64;384,76,80,64,32;390,76,80,32,64;384,76,80,32,64"
for s in 1 2; do
  APPLESTAR_CONV_V2_NARROW_SUB=$s timeout -k 10 200 python tools/bench_conv_psb.py 20 v2 > gpurun_out/s19_conv_sub$s.jsonl 2>/dev/null || exit 1
  echo "sub=$s"; cat gpurun_out/s19_conv_sub$s.jsonl
done
unset CONV_SHAPES
for i in 1 2; do
  for s in 2 1; do
    APPLESTAR_CONV_V2_NARROW_SUB=$s timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s19_fp32_sub${s}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s19_fp32_sub${s}_$i.json'));print('fp32 narrow_sub=$s', $i, d['ms_per_step'])"
  done
done
