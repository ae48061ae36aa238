# step_graph: does the round-2 split-LSTM poll budget (2^16, 'shortpoll' variant) reproduce the graph failure
# without host waits?  + the graph test and a graphed bf16 bench without host waits on the release build
O=gpurun_out/r3l; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
SP=$PWD/$(ls diag_ext/_C*.so)
step sp_alone_nosync 240 env STEPS=12 APPLESTAR_EXT_PATH=$SP python -u tools/diag/graph_sync_diag.py alone > $O/sp_alone_nosync.jsonl 2> $O/sp_alone_nosync.err
step sp_inter_nosync 240 env STEPS=12 APPLESTAR_EXT_PATH=$SP python -u tools/diag/graph_sync_diag.py interleaved > $O/sp_inter_nosync.jsonl 2> $O/sp_inter_nosync.err
step sp_alone_sync 240 env STEPS=12 APPLESTAR_GRAPH_HOST_SYNC=1 APPLESTAR_EXT_PATH=$SP python -u tools/diag/graph_sync_diag.py alone > $O/sp_alone_sync.jsonl 2> $O/sp_alone_sync.err
step rel_alone_nosync 240 env STEPS=12 python -u tools/diag/graph_sync_diag.py alone > $O/rel_alone_nosync.jsonl 2> $O/rel_alone_nosync.err
step test_graph_nosync 300 env APPLESTAR_GRAPH_HOST_SYNC=0 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_model_gpu.py -k graphed > $O/test_graph_nosync.txt 2>&1
step bench_graph_nosync 300 env APPLESTAR_GRAPH_HOST_SYNC=0 python -u bench.py --precision bf16 --graph --steps 10 --warmup 4 > $O/bench_graph_nosync.json 2> $O/bench_graph_nosync.err
step bench_graph_sync 300 python -u bench.py --precision bf16 --graph --steps 10 --warmup 4 > $O/bench_graph_sync.json 2> $O/bench_graph_sync.err
echo done >> $O/progress.txt
