set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_parity_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "bf16_gpu_vs_cpu or head_grad_error" -s > gpurun_out/r5f_parity.txt 2>&1; echo "parity rc=$?"
grep -E "passed|failed" gpurun_out/r5f_parity.txt | tail -2
timeout -k 10 300 python -u tools/glue_sites.py --steps 2 --timed --top 45 > gpurun_out/r5f_glue_timed.txt 2>&1 || { tail -30 gpurun_out/r5f_glue_timed.txt; exit 1; }
grep -A 60 "event-timed" gpurun_out/r5f_glue_timed.txt | cut -c1-200
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5e_bench_fp32.json 2> gpurun_out/r5e_bench_fp32.log || exit 1
cat gpurun_out/r5e_bench_fp32.json
timeout -k 10 900 python -u -m pytest tests/test_learning_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r5e_learning_pytest.txt 2>&1 || { tail -30 gpurun_out/r5e_learning_pytest.txt; exit 1; }
tail -3 gpurun_out/r5e_learning_pytest.txt
cd /tmp && export TMPDIR=/tmp
for B in 1 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5e_inf_b$B -o run --output-format csv -- python3 $R/tools/bench_inference.py --batches $B --iters 40 --graphs 1 > $R/gpurun_out/r5e_inf_b$B.log 2>&1 || exit 1
  f=$(find $R/gpurun_out/r5e_inf_b$B -name '*kernel_stats.csv' -print -quit)
  cp $f $R/gpurun_out/r5e_inf_b${B}_kernel_stats.csv
  t=$(find $R/gpurun_out/r5e_inf_b$B -name '*kernel_trace.csv' -print -quit)
  cp $t $R/gpurun_out/r5e_inf_b${B}_kernel_trace.csv
  rm -rf $R/gpurun_out/r5e_inf_b$B
  tail -4 $R/gpurun_out/r5e_inf_b$B.log
done
cd $R
timeout -k 10 300 python tools/rl_train_dp_rehearsal.py --iters 8 --out gpurun_out/r5e_rl_train_dp2 --timeout 280 > gpurun_out/r5e_dp2.json 2>&1 || { tail -5 gpurun_out/r5e_dp2.json; tail -20 gpurun_out/r5e_rl_train_dp2/learner.log; exit 1; }
tail -1 gpurun_out/r5e_dp2.json
for i in 1 2 3; do
  timeout -k 10 200 python tools/actor_step_profile.py --steps 600 >> gpurun_out/r5e_actor_cpu.jsonl 2>&1 || exit 1
done
cat gpurun_out/r5e_actor_cpu.jsonl
