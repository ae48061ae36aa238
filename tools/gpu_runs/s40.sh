set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in base padded; do
    case $v in base) E="";; padded) E="APPLESTAR_PACKED_SCATTER=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s40_bf16_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s40_bf16_${v}_$i.json'));m=d.get('mixed_bf16',d);print('bf16 $v', $i, d['ms_per_step'], m.get('step_ms_median'), m.get('host_ms_per_step'))"
  done
done
