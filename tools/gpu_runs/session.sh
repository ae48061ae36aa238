set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv3x3_f32 or gemm_f32 or linear" > gpurun_out/prio_pytest.txt 2>&1 || { tail -40 gpurun_out/prio_pytest.txt; exit 1; }
tail -1 gpurun_out/prio_pytest.txt
APPLESTAR_PIPE_PRIO=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv3x3_f32 or gemm_f32" > gpurun_out/prio1_pytest.txt 2>&1 || { tail -40 gpurun_out/prio1_pytest.txt; exit 1; }
tail -1 gpurun_out/prio1_pytest.txt
APPLESTAR_PIPE_PRIO=1 timeout -k 10 200 python -u tools/bench_f32_kernels.py conv > gpurun_out/prio1_conv.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_f32_kernels.py conv > gpurun_out/prio0_conv.jsonl 2>&1 || exit 1
paste -d' ' <(grep -o '"shape": \[[^]]*\], "us": [0-9.]*' gpurun_out/prio1_conv.jsonl) <(grep -o '"us": [0-9.]*' gpurun_out/prio0_conv.jsonl)
for i in 1 2; do
  APPLESTAR_PIPE_PRIO=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/prio1_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/prio1_f32_$i.json'));print('fp32 prio', $i, d['ms_per_step'])"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/prio0_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/prio0_f32_$i.json'));print('fp32 default', $i, d['ms_per_step'])"
done
