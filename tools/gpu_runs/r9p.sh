set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r9p_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r9p_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r9p_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r9p_trace --last 600 > gpurun_out/r9p_timeline_b1_policy_graph.txt && grep -c . gpurun_out/r9p_timeline_b1_policy_graph.txt
