set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_derived_weights_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "su_sample or fused_gated or cached_forms or resmlp_fused" > gpurun_out/r5u_pytest_focus.txt 2>&1; rc=$?
tail -3 gpurun_out/r5u_pytest_focus.txt; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r5u_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5u_bench_inference.jsonl | cut -c1-300
APPLESTAR_GRAPH_SIDE_STREAMS=1 timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph > gpurun_out/r5u_bench_inference_side.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r5u_bench_inference_side.jsonl | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5u_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r5u_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r5u_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r5u_trace --last 600 > gpurun_out/r5u_timeline_b1_policy_graph.txt && head -3 gpurun_out/r5u_timeline_b1_policy_graph.txt && tail -1 gpurun_out/r5u_timeline_b1_policy_graph.txt
APPLESTAR_PIPE_PROFILE_AT=25 APPLESTAR_PIPE_PROFILE_N=5 APPLESTAR_PIPE_PROFILE_OUT=$PWD/gpurun_out/r5u_learner_profile.txt timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_32 > gpurun_out/r5u_pipeline_envs32.json 2> gpurun_out/r5u_pipeline_envs32.log || { tail -20 gpurun_out/r5u_pipeline_envs32.log; exit 1; }
head -45 gpurun_out/r5u_learner_profile.txt
