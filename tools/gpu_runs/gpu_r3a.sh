# round-3 GPU session: cold bf16 bench first, fp32 attention numerics, whole-model parity, diag, both-precision
# bench, rocprof stats.  Test failures (rc 1) do not stop the session; anything else (fault, timeout) does.
O=gpurun_out/r3a; mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
(nproc; lscpu | grep -i "model name"; uptime; free -g) > $O/host.txt 2>&1
step bench_bf16_first 300 python -u bench.py --precision bf16 --steps 20 --warmup 5 --inference 0 > $O/bench_bf16_first.json 2> $O/bench_bf16_first.err
step pytest_attn 240 python -u -m pytest tests/test_kernels_gpu.py -k "varlen" -x -v --timeout 120 --timeout-method thread > $O/pytest_attn.txt 2>&1
step pytest_parity 600 python -u -m pytest tests/test_model_parity_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_parity.txt 2>&1
cp gpurun_out/*.json $O/ 2>/dev/null
step layer_diag 300 python -u tools/diag/layer_grad_diag.py > $O/layer_grad_diag.txt 2>&1
step bench_both 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_both.json 2> $O/bench_both.err
P=/tmp/r3a_prof; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/$O
step rocprof_bf16 300 rocprofv3 --kernel-trace --stats -d $P/bf16 -o run -- python $R/bench.py --precision bf16 --steps 10 --warmup 5 --inference 0 > $O/prof_bf16.log 2>&1
find $P/bf16 -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_bf16.csv \;
step rocprof_fp32 400 rocprofv3 --kernel-trace --stats -d $P/fp32 -o run -- python $R/bench.py --precision fp32 --steps 5 --warmup 3 --inference 0 > $O/prof_fp32.log 2>&1
find $P/fp32 -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_fp32.csv \;
echo done >> $O/progress.txt
