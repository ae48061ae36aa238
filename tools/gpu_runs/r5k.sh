set -o pipefail
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u -m pytest tests/test_glue_fusions_gpu.py -m gpu -v --timeout 200 --timeout-method thread -k "entity_pack or col_assemble or embed_relu" > gpurun_out/r5k_glue_pytest.txt 2>&1; rc=$?
grep -E "PASS|FAIL|^E " gpurun_out/r5k_glue_pytest.txt | head -20; ok $rc || exit 1
for v in default nopost noemb nocol; do
  case $v in default) E="";; nopost) E="APPLESTAR_POST_ADD=0";; noemb) E="APPLESTAR_EMBED_RELU=0";; nocol) E="APPLESTAR_COL_ASSEMBLE=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5k_bench_$v.json 2> gpurun_out/r5k_bench_$v.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r5k_bench_$v.json'));print('$v', d['ms_per_step'])"
done
timeout -k 10 200 python -u tools/inference_casts.py --batch 1 --top 70 > gpurun_out/r5k_inference_casts.txt 2>&1 || { tail -20 gpurun_out/r5k_inference_casts.txt; exit 1; }
head -40 gpurun_out/r5k_inference_casts.txt
timeout -k 10 300 python tools/rl_train_dp_rehearsal.py --iters 8 --out /tmp/r5k_dp2 --timeout 280 > gpurun_out/r5k_dp2.json 2>&1; rc=$?
mkdir -p gpurun_out/r5k_dp2_logs && cp /tmp/r5k_dp2/*.log gpurun_out/r5k_dp2_logs/ 2>/dev/null
tail -2 gpurun_out/r5k_dp2.json; echo "dp rc=$rc"
grep -n -E "Error|Traceback" gpurun_out/r5k_dp2_logs/learner.log | head -10
