# autograd node attribution (fp32 + bf16 steps) and a bf16 steady-state kernel profile
O=gpurun_out/r3m; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step nodes_fp32 300 python -u tools/diag/autograd_nodes.py --precision fp32 > $O/autograd_nodes_fp32.txt 2> $O/nodes_fp32.err
step nodes_bf16 300 python -u tools/diag/autograd_nodes.py --precision bf16 > $O/autograd_nodes_bf16.txt 2> $O/nodes_bf16.err
step prof_bf16 400 env TAG=r3m_bf16 ITERS=7 STEADY=3 PROF_TIMEOUT=350 BENCH_ARGS="--precision bf16 --steps 4 --warmup 3 --inference 0" bash tools/gpu_prof.sh > $O/prof_bf16.out 2>&1
echo done >> $O/progress.txt
