set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/s2_pytest_wgrad.txt 2>&1 || { tail -40 gpurun_out/s2_pytest_wgrad.txt; exit 1; }
tail -1 gpurun_out/s2_pytest_wgrad.txt
APPLESTAR_WGRAD_STG_NARROW=0 timeout -k 10 200 python tools/bench_wgrad32.py > gpurun_out/s2_wgrad32_off.jsonl 2>/dev/null || exit 1
timeout -k 10 200 python tools/bench_wgrad32.py > gpurun_out/s2_wgrad32_on.jsonl 2>/dev/null || exit 1
paste -d' ' <(python -c "import json;[print(d['shape'],d['us'],d['tflops']) for d in map(json.loads,open('gpurun_out/s2_wgrad32_off.jsonl'))]") <(python -c "import json;[print(d['us'],d['tflops'],d['err_max']) for d in map(json.loads,open('gpurun_out/s2_wgrad32_on.jsonl'))]")
for i in 1 2; do
  for m in 1 0; do
    APPLESTAR_WGRAD_STG_NARROW=$m timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s2_fp32_n${m}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s2_fp32_n${m}_$i.json'));print('narrow=$m', $i, d['ms_per_step'])"
  done
done
for i in 1 2; do
  for r in 96 0; do
    APPLESTAR_WGRAD_SMALL_R=$r timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s2_fp32_sr${r}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s2_fp32_sr${r}_$i.json'));print('small_r=$r', $i, d['ms_per_step'])"
  done
done
