set -o pipefail
mkdir -p gpurun_out
for cfg in "32 -1" "32 0" "64 -1"; do
  set -- $cfg; E=$1; P=$2
  APPLESTAR_INFERENCE_STREAM_PRIORITY=$P timeout -k 10 240 python -u tools/bench_pipeline.py --envs $E --seconds 40 --precision fp32 --workdir /tmp/pipe_${E}_$P > gpurun_out/r5h_pipeline_envs${E}_prio$P.json 2> gpurun_out/r5h_pipeline_envs${E}_prio$P.log || { tail -20 gpurun_out/r5h_pipeline_envs${E}_prio$P.log; exit 1; }
  tail -c 1200 gpurun_out/r5h_pipeline_envs${E}_prio$P.json; echo
done
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_flat_model.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r5h_inf_pytest.txt 2>&1; echo "inf tests rc=$?"; tail -3 gpurun_out/r5h_inf_pytest.txt
timeout -k 10 200 python -u tools/inference_casts.py --batch 1 --top 40 > gpurun_out/r5h_inference_casts.txt 2>&1 || exit 1
head -45 gpurun_out/r5h_inference_casts.txt
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 40 > gpurun_out/r5h_bench_inference.jsonl 2>&1 || exit 1
cat gpurun_out/r5h_bench_inference.jsonl
