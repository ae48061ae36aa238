set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  for v in base nofold; do
    case $v in base) E="";; nofold) E="APPLESTAR_SU_FOLD=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/s35_bf16_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s35_bf16_${v}_$i.json'));print('bf16 $v', $i, d['ms_per_step'])"
  done
done
