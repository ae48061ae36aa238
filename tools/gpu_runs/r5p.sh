set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_model_parity_gpu.py tests/test_kernels_gpu.py -m gpu -q --timeout 200 --timeout-method thread -k "psb or fp32 or deferred or gated" > gpurun_out/r5p_pytest.txt 2>&1; rc=$?
grep -E "passed|failed|^E |FAIL" gpurun_out/r5p_pytest.txt | head -12; ok $rc || exit 1
for v in default nopsb; do
  case $v in default) E="";; nopsb) E="APPLESTAR_GEMM_PSB=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5p_bench_$v.json 2> gpurun_out/r5p_bench_$v.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r5p_bench_$v.json'));print('$v', d['ms_per_step'])"
done
APPLESTAR_LSTM_SPLIT=0 timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_ns > gpurun_out/r5p_pipeline_envs32_nosplit.json 2> gpurun_out/r5p_pipeline_envs32_nosplit.log || { tail -20 gpurun_out/r5p_pipeline_envs32_nosplit.log; exit 1; }
tail -c 1500 gpurun_out/r5p_pipeline_envs32_nosplit.json
