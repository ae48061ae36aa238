set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --mode sl --steps 20 --warmup 5 --precision fp32 > gpurun_out/r4z_bench_sl.json 2> gpurun_out/r4z_bench_sl.err || { tail -20 gpurun_out/r4z_bench_sl.err; exit 1; }
tail -1 gpurun_out/r4z_bench_sl.json
