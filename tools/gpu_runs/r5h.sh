set -o pipefail
mkdir -p gpurun_out
for cfg in "32 -1" "32 0" "64 -1"; do
  set -- $cfg; E=$1; P=$2
  APPLESTAR_INFERENCE_STREAM_PRIORITY=$P timeout -k 10 240 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_${E}_$P > gpurun_out/r5h_pipeline_envs${E}_prio$P.json 2> gpurun_out/r5h_pipeline_envs${E}_prio$P.log || { tail -20 gpurun_out/r5h_pipeline_envs${E}_prio$P.log; exit 1; }
  tail -c 1200 gpurun_out/r5h_pipeline_envs${E}_prio$P.json; echo
done
