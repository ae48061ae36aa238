set -o pipefail
mkdir -p gpurun_out
b() {  # name, env..., then bench args via BARGS
  N=$1; shift
  env "$@" timeout -k 10 400 python bench.py --precision fp32 --inference 0 $BARGS > gpurun_out/r5z_bench_$N.json 2> gpurun_out/r5z_bench_$N.log || { tail -5 gpurun_out/r5z_bench_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r5z_bench_$N.json'));print('$N', d['ms_per_step'])"
}
BARGS="--steps 10 --warmup 3 --n-batches 2" b fixed2 A=1 || exit 1
BARGS="--steps 10 --warmup 3 --n-batches 13" b fresh13 A=1 || exit 1
BARGS="--steps 10 --warmup 3 --n-batches 13" b fresh13_rocblas TORCH_BLAS_PREFER_HIPBLASLT=0 || exit 1
BARGS="--steps 10 --warmup 13 --n-batches 13" b seen13 A=1 || exit 1
