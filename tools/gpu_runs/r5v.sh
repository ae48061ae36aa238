set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/r5v_trace -o run -- python $GRAFT_REPO_ROOT/tools/bench_inference.py --batches 1 --iters 5 --modes policy_graph > /tmp/r5v_trace.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r5v_trace.log; exit 1; }
python tools/trace_timeline.py /tmp/r5v_trace --last 700 > gpurun_out/r5v_timeline_b1_policy_graph.txt && head -2 gpurun_out/r5v_timeline_b1_policy_graph.txt && tail -1 gpurun_out/r5v_timeline_b1_policy_graph.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5v_bench_alone.json 2> gpurun_out/r5v_bench_alone.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/r5v_bench_alone.json'));print('alone', d['ms_per_step'])"
timeout -k 10 200 python tools/bench_inference.py --batches 16 --iters 40000 --modes policy_graph > gpurun_out/r5v_bg_inference.log 2>&1 &
BG=$!
sleep 45
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5v_bench_corun.json 2> gpurun_out/r5v_bench_corun.log; rc=$?
kill $BG 2>/dev/null; wait $BG 2>/dev/null
[ $rc -eq 0 ] || exit 1
python -c "import json;d=json.load(open('gpurun_out/r5v_bench_corun.json'));print('with inference loop', d['ms_per_step'])"
APPLESTAR_PIPE_PROFILE_AT=25 APPLESTAR_PIPE_PROFILE_N=5 APPLESTAR_PIPE_PROFILE_OUT=$PWD/gpurun_out/r5v_learner_profile.txt timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_32 > gpurun_out/r5v_pipeline_envs32.json 2> gpurun_out/r5v_pipeline_envs32.log || { tail -20 gpurun_out/r5v_pipeline_envs32.log; exit 1; }
head -25 gpurun_out/r5v_learner_profile.txt
