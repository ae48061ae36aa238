set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_glue_fusions_gpu.py -m gpu -q --timeout 100 --timeout-method thread -k "psb" > gpurun_out/r5r_pytest.txt 2>&1; rc=$?
grep -E "passed|failed|^E |FAIL" gpurun_out/r5r_pytest.txt | head -8; ok $rc || exit 1
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 100 --timeout-method thread -k "fused_gated_resblock" > gpurun_out/r5r_gated_alone.txt 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r5r_gated_alone.txt; ok $rc || exit 1
for v in both none both2 none2; do
  case $v in both|both2) E="";; none|none2) E="APPLESTAR_GEMM_PSB=0 APPLESTAR_CONV_PSB=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5r_bench_$v.json 2> gpurun_out/r5r_bench_$v.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r5r_bench_$v.json'));print('$v', d['ms_per_step'])"
done
timeout -k 10 240 python -u tools/bench_pipeline.py --envs 32 --seconds 40 --precision fp32 --workdir /tmp/pipe_h > gpurun_out/r5r_pipeline_envs32.json 2> gpurun_out/r5r_pipeline_envs32.log || { tail -20 gpurun_out/r5r_pipeline_envs32.log; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r5r_pipeline_envs32.json'));print({k: d[k] for k in ('learner_iters_per_s','learner_train_ms_mean','learner_train_host_ms_mean','learner_iter_ms_mean','fresh_samples_per_s')})"
