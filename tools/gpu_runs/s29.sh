set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base vebwd vefirst; do
    case $v in base) E="";; vebwd) E="APPLESTAR_VE_BWD_OVERLAP=1";; vefirst) E="APPLESTAR_VE_AFTER_CORE=0";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s29_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s29_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
  done
done
