set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/r6q_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r6q_pytest_gpu.txt; [ $rc -eq 0 ] || exit 1
for R in 1 2; do
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r6q_bench_inference_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r6q_bench_inference_$R.jsonl | cut -c1-200
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6q_smoke.txt 2>&1 || { tail -5 gpurun_out/r6q_smoke.txt; exit 1; }
tail -1 gpurun_out/r6q_smoke.txt
