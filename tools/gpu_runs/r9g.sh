set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "su_sample or graphed_policy or inference or policy" > gpurun_out/r9g_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r9g_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r9g_pytest.txt | head; exit 1; }
for R in 1 2; do
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r9g_bench_inference_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r9g_bench_inference_$R.jsonl | cut -c1-200
done
