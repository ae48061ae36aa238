# where the host waits in the fp32 / bf16 learner step: sync points and host phase times (pipelined)
O=gpurun_out/r3s; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  echo "$(date +%T) $name" >> $O/progress.txt
  timeout -k 10 $t "$@"; local rc=$?
  echo "$(date +%T) $name rc=$rc" >> $O/progress.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step sync_fp32 200 python -u tools/sync_points.py --fp32 > $O/sync_fp32.txt 2>&1
step sync_bf16 200 python -u tools/sync_points.py > $O/sync_bf16.txt 2>&1
step phases_fp32 200 python -u tools/host_phases.py --fp32 --batch 6 --unroll 64 --max-entities 512 --steps 6 --no-sync > $O/phases_fp32.txt 2>&1
step phases_fp32_sync 200 python -u tools/host_phases.py --fp32 --batch 6 --unroll 64 --max-entities 512 --steps 6 > $O/phases_fp32_sync.txt 2>&1
step phases_bf16 200 python -u tools/host_phases.py --batch 6 --unroll 64 --max-entities 512 --steps 6 --no-sync > $O/phases_bf16.txt 2>&1
step phases_bf16_small 200 python -u tools/host_phases.py --steps 6 > $O/phases_bf16_small.txt 2>&1
echo done >> $O/progress.txt
