set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_glue_fusions_gpu.py tests/test_model_parity_gpu.py tests/test_model_gpu.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r6h_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r6h_pytest.txt; [ $rc -eq 0 ] || exit 1
b() {  # name precision env...
  N=$1; P=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision $P --inference 0 > gpurun_out/r6h_bench_$N.json 2> gpurun_out/r6h_bench_$N.log || { tail -5 gpurun_out/r6h_bench_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6h_bench_$N.json'));print('$N', d['ms_per_step'], 'host', d['config'].get('host_ms_per_step'))"
}
b bf16_fast bf16 APPLESTAR_FAST_APPLY=1 || exit 1
b bf16_slow bf16 APPLESTAR_FAST_APPLY=0 || exit 1
b bf16_fast2 bf16 APPLESTAR_FAST_APPLY=1 || exit 1
b bf16_slow2 bf16 APPLESTAR_FAST_APPLY=0 || exit 1
b fp32_fast fp32 APPLESTAR_FAST_APPLY=1 || exit 1
b fp32_slow fp32 APPLESTAR_FAST_APPLY=0 || exit 1
