set -o pipefail
mkdir -p gpurun_out
b() {  # name precision env...
  N=$1; P=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision $P --inference 0 $BARGS > gpurun_out/r6e_bench_$N.json 2> gpurun_out/r6e_bench_$N.log || { tail -5 gpurun_out/r6e_bench_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6e_bench_$N.json'));print('$N', d['ms_per_step'])"
}
BARGS="--graph" b bf16_graph bf16 A=1 || exit 1
BARGS="--graph" b fp32_graph fp32 A=1 || exit 1
timeout -k 10 400 python -u tools/glue_sites.py --precision fp32 --timed --premask --top 50 > gpurun_out/r6e_glue_fp32.txt 2>&1 || { tail -5 gpurun_out/r6e_glue_fp32.txt; exit 1; }
grep -A25 "ReLU backward passes" gpurun_out/r6e_glue_fp32.txt
