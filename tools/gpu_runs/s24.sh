set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base g12 g14 a7 a31; do
    case $v in base) E="";; g12) E="APPLESTAR_GEMM_PSB_VARIANT=12";; g14) E="APPLESTAR_GEMM_PSB_VARIANT=14";; a7) E="APPLESTAR_F32_ATTN_IMG=7";; a31) E="APPLESTAR_F32_ATTN_IMG=31";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s24_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s24_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
  done
done
