set -o pipefail
mkdir -p gpurun_out
cat /proc/loadavg
OFF="APPLESTAR_HEAD_LOGITS_SIDE=0 APPLESTAR_SU_SIDE_STREAM=0 APPLESTAR_TU_SIDE_STREAM=0 APPLESTAR_SU_AE_SIDE=0 APPLESTAR_SMALL_TN_WAVES=4"
for i in 1 2 3; do
  for v in new off; do
    case $v in new) E="";; off) E="$OFF";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s16_bf16_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s16_bf16_${v}_$i.json'));print('bf16 $v', $i, d['ms_per_step'], 'host', d.get('host_ms_per_step'), 'min/med/max', d.get('step_ms_min'), d.get('step_ms_median'), d.get('step_ms_max'))"
  done
  cat /proc/loadavg
done
