set -o pipefail
mkdir -p gpurun_out
b() {  # name precision env...
  N=$1; P=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision $P --inference 0 $BARGS > gpurun_out/r6d_bench_$N.json 2> gpurun_out/r6d_bench_$N.log || { tail -5 gpurun_out/r6d_bench_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6d_bench_$N.json'));print('$N', d['ms_per_step'])"
}
b fp32_base fp32 A=1 || exit 1
b fp32_pipe4 fp32 APPLESTAR_LSTM_PIPELINE=4 || exit 1
b fp32_pipe2 fp32 APPLESTAR_LSTM_PIPELINE=2 || exit 1
b bf16_base bf16 A=1 || exit 1
b bf16_pipe4 bf16 APPLESTAR_LSTM_PIPELINE=4 || exit 1
BARGS="--graph" b bf16_graph bf16 A=1 || exit 1
BARGS="--graph" b fp32_graph fp32 A=1 || exit 1
