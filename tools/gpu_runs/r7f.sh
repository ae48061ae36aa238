set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_model_parity_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "graphed_policy or inference_server or su_sample or head_sample or policy or parity or bf16 or scalar or encoder or target_unit" > gpurun_out/r7f_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r7f_pytest.txt; [ $rc -eq 0 ] || exit 1
for R in 1 2; do
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r7f_bench_inference_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r7f_bench_inference_$R.jsonl | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r7f_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r7f_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r7f_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r7f_trace --last 600 > gpurun_out/r7f_timeline_b1_policy_graph.txt && grep -c . gpurun_out/r7f_timeline_b1_policy_graph.txt
