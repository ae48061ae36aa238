# end-to-end pipeline with the learner in its own process (bf16 and fp32), 12 env workers
O=gpurun_out/r3q; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pipeline_bf16 300 python -u tools/bench_pipeline.py --envs 12 --seconds 60 --batch 6 --traj-len 64 > $O/pipeline_bf16.json 2> $O/pipeline_bf16.err
step pytest_shared 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_gpu.py -k "shared_batch" > $O/pytest_shared.txt 2>&1
echo done >> $O/progress.txt
