set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 420 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/r6a_trace -o run_%pid% -- python $GRAFT_REPO_ROOT/tools/bench_pipeline.py --envs 8 --seconds 20 --precision fp32 --workdir /tmp/pipe_8 > /tmp/r6a_pipe.json 2> /tmp/r6a_pipe.log; rc=$?; cd $GRAFT_REPO_ROOT
cp /tmp/r6a_pipe.json gpurun_out/r6a_pipeline_envs8_traced.json 2>/dev/null
[ $rc -eq 0 ] || { tail -20 /tmp/r6a_pipe.log; exit 1; }
cp /tmp/r6a_pipe.log gpurun_out/r6a_pipe.log; find /tmp/r6a_trace -name "*.csv" | head -20
python tools/pipeline_trace_summary.py /tmp/r6a_trace > gpurun_out/r6a_pipeline_trace_summary.txt 2>&1; cat gpurun_out/r6a_pipeline_trace_summary.txt | head -80
