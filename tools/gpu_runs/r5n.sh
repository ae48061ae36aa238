set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_gemm_psb.py 20 > gpurun_out/r5n_gemm_psb.jsonl 2>&1; rc=$?
cat gpurun_out/r5n_gemm_psb.jsonl; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --graph-step --workdir /tmp/pipe_g > gpurun_out/r5n_pipeline_envs32_graph.json 2> gpurun_out/r5n_pipeline_envs32_graph.log || { tail -20 gpurun_out/r5n_pipeline_envs32_graph.log; exit 1; }
tail -c 1500 gpurun_out/r5n_pipeline_envs32_graph.json
