set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_model_parity_gpu.py tests/test_glue_fusions_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "multi_copy or scalar or encoder or parity or policy or graphed or inference" > gpurun_out/r9o_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r9o_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r9o_pytest.txt | head; exit 1; }
for R in 1 2; do
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r9o_bench_inference_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r9o_bench_inference_$R.jsonl | cut -c1-200
done
timeout -k 10 300 python -u bench.py --precision fp32 --sl 0 > gpurun_out/r9o_bench.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r9o_bench.json')); print(d['ms_per_step'], d.get('inference_p50_ms'))"
