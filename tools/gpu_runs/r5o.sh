set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 200 python -u -m pytest tests/test_glue_fusions_gpu.py -m gpu -q --timeout 100 --timeout-method thread -k "psb or logp" > gpurun_out/r5o_pytest.txt 2>&1; rc=$?
grep -E "passed|failed|^E |FAIL" gpurun_out/r5o_pytest.txt | head -12; ok $rc || exit 1
timeout -k 10 200 python -u tools/bench_gemm_psb.py 20 > gpurun_out/r5o_gemm_psb.jsonl 2>&1; rc=$?
grep -E "kernel|presplit" gpurun_out/r5o_gemm_psb.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --graph-step --workdir /tmp/pipe_g > gpurun_out/r5o_pipeline_envs32_graph.json 2> gpurun_out/r5o_pipeline_envs32_graph.log || { tail -20 gpurun_out/r5o_pipeline_envs32_graph.log; exit 1; }
tail -c 1500 gpurun_out/r5o_pipeline_envs32_graph.json
