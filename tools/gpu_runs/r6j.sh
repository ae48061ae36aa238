set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "conv3x3 or graphed_policy or inference_server" > gpurun_out/r6j_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r6j_pytest.txt; [ $rc -eq 0 ] || exit 1
for V in 1 0 1; do
APPLESTAR_CONV_SMALLM=$V timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r6j_bench_inference_smallm$V.jsonl 2>&1 || exit 1
echo "smallm=$V"; grep -v amdgpu.ids gpurun_out/r6j_bench_inference_smallm$V.jsonl | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r6j_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r6j_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r6j_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r6j_trace --last 420 > gpurun_out/r6j_timeline_b1_policy_graph.txt && head -2 gpurun_out/r6j_timeline_b1_policy_graph.txt
