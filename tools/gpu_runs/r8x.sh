set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv3x3" > gpurun_out/r8x_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8x_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8x_pytest.txt | head; exit 1; }
for R in 1 2; do
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r8x_bench_inference_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r8x_bench_inference_$R.jsonl | cut -c1-200
APPLESTAR_CONV_RING=0 timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r8x_bench_inference_ring0_$R.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r8x_bench_inference_ring0_$R.jsonl | cut -c1-200
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r8x_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r8x_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r8x_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r8x_trace --last 600 > gpurun_out/r8x_timeline_b1_policy_graph.txt && grep -c . gpurun_out/r8x_timeline_b1_policy_graph.txt
grep -E "conv3x3" gpurun_out/r8x_timeline_b1_policy_graph.txt | head -5 | cut -c1-120
