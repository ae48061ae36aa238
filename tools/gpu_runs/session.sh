set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "varlen_attention" > gpurun_out/attn_pytest.txt 2>&1 || { tail -30 gpurun_out/attn_pytest.txt; exit 1; }
tail -2 gpurun_out/attn_pytest.txt
timeout -k 10 200 python -u tools/bench_f32_kernels.py attn > gpurun_out/attn_micro.jsonl 2>&1 || { tail -20 gpurun_out/attn_micro.jsonl; exit 1; }
cat gpurun_out/attn_micro.jsonl
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/attn_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/attn_f32_$i.json'));print('fp32', $i, d['ms_per_step'])"
  APPLESTAR_F32_ATTN_IMG=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/attn0_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/attn0_f32_$i.json'));print('fp32 perwave', $i, d['ms_per_step'])"
done
