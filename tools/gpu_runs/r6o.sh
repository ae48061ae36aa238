set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "graphed_policy or inference_server or su_sample or head_sample or policy" > gpurun_out/r6o_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r6o_pytest.txt; [ $rc -eq 0 ] || exit 1
for R in 1 2; do
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r6o_bench_inference_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r6o_bench_inference_$R.jsonl | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r6o_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r6o_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r6o_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r6o_trace --last 600 > gpurun_out/r6o_timeline_b1_policy_graph.txt && grep su_sample gpurun_out/r6o_timeline_b1_policy_graph.txt | cut -c1-60
timeout -k 10 200 python -u tools/inference_casts.py --batch 1 --top 60 > gpurun_out/r6o_inference_ops_b1.txt 2>&1 || exit 1
head -4 gpurun_out/r6o_inference_ops_b1.txt
