set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }   # 1 = test assertions failed (GPU fine): go on; anything else: stop
timeout -k 10 300 python -u -m pytest tests/test_glue_fusions_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r5j_glue_pytest.txt 2>&1; rc=$?
grep -E "PASS|FAIL|^E " gpurun_out/r5j_glue_pytest.txt | head -20; ok $rc || exit 1
timeout -k 10 400 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -v --timeout 300 --timeout-method thread -k "bf16_gpu_vs_cpu or head_grad_error" -s > gpurun_out/r5j_parity.txt 2>&1; rc=$?
grep -E "PASS|FAIL|^E " gpurun_out/r5j_parity.txt | head -20; ok $rc || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5j_bench_fp32.json 2> gpurun_out/r5j_bench_fp32.log || exit 1
cat gpurun_out/r5j_bench_fp32.json
timeout -k 10 300 python -u tools/glue_sites.py --steps 2 --timed --premask --top 100 > gpurun_out/r5j_glue_timed.txt 2>&1 || { tail -30 gpurun_out/r5j_glue_timed.txt; exit 1; }
grep -A 30 "not folded" gpurun_out/r5j_glue_timed.txt
timeout -k 10 300 python tools/rl_train_dp_rehearsal.py --iters 8 --out /tmp/r5j_dp2 --timeout 280 > gpurun_out/r5j_dp2.json 2>&1; rc=$?
mkdir -p gpurun_out/r5j_dp2_logs && cp /tmp/r5j_dp2/*.log gpurun_out/r5j_dp2_logs/ 2>/dev/null
tail -2 gpurun_out/r5j_dp2.json; echo "dp rc=$rc"
grep -n -E "Error|error|Traceback|raise" gpurun_out/r5j_dp2_logs/learner.log | head -20
cd /tmp && export TMPDIR=/tmp
for B in 1 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r5j_inf_b$B -o run --output-format csv -- python3 $R/tools/bench_inference.py --batches $B --iters 40 --graphs 1 > $R/gpurun_out/r5j_inf_b$B.log 2>&1 || exit 1
  f=$(find /tmp/r5j_inf_b$B -name '*kernel_stats.csv' -print -quit)
  cp $f $R/gpurun_out/r5j_inf_b${B}_kernel_stats.csv
  t=$(find /tmp/r5j_inf_b$B -name '*kernel_trace.csv' -print -quit)
  gzip -c $t > $R/gpurun_out/r5j_inf_b${B}_kernel_trace.csv.gz
  tail -4 $R/gpurun_out/r5j_inf_b$B.log
done
du -sh $R/gpurun_out
