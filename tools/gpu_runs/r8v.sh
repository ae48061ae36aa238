set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r8v_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r8v_bench_inference.jsonl | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r8v_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r8v_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r8v_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r8v_trace --last 600 > gpurun_out/r8v_timeline_b1_policy_graph.txt && grep -c . gpurun_out/r8v_timeline_b1_policy_graph.txt
grep -E "su_sample|conv3x3" gpurun_out/r8v_timeline_b1_policy_graph.txt | head -30 | cut -c1-120
