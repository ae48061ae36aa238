set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "varlen or graphed or inference" > gpurun_out/r5m_pytest.txt 2>&1; rc=$?
grep -E "passed|failed|^E |FAIL" gpurun_out/r5m_pytest.txt | head -12; ok $rc || exit 1
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 40 > gpurun_out/r5m_bench_inference.jsonl 2>&1 || exit 1
cat gpurun_out/r5m_bench_inference.jsonl
timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_32 > gpurun_out/r5m_pipeline_envs32.json 2> gpurun_out/r5m_pipeline_envs32.log || { tail -20 gpurun_out/r5m_pipeline_envs32.log; exit 1; }
tail -c 1500 gpurun_out/r5m_pipeline_envs32.json
