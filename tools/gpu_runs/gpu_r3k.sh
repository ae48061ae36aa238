# step_graph host-wait root cause: graphed trainer without host waits, four variants + a kernel trace
O=gpurun_out/r3k; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
for v in interleaved alone private_pools presync; do
  step diag_$v 240 python -u tools/diag/graph_sync_diag.py $v > $O/graph_sync_$v.jsonl 2> $O/graph_sync_$v.err
done
R=$PWD
step trace 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --output-format csv -d /tmp/gs -o run -- python3 $R/tools/diag/graph_sync_diag.py alone > $R/$O/trace_run.jsonl 2>&1"
f=$(find /tmp/gs -name '*kernel_trace.csv' | head -1); [ -n "$f" ] && gzip -c "$f" > $O/graph_kernel_trace.csv.gz
echo done >> $O/progress.txt
