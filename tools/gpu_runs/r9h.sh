set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in 32 64; do
timeout -k 10 300 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_$E > gpurun_out/r9h_pipeline_envs$E.json 2> gpurun_out/r9h_pipeline_envs$E.log || { tail -20 gpurun_out/r9h_pipeline_envs$E.log; exit 1; }
cut -c1-900 gpurun_out/r9h_pipeline_envs$E.json
done
