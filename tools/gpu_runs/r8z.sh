set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# two ranks sharing the one GPU over gloo: the multi-rank bench path (two-phase backward, bucketed all-reduce,
# bf16 master-weight wire) on real kernels
APPLESTAR_DIST_BACKEND=gloo timeout -k 20 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --inference 0 --sl 0 > gpurun_out/r8z_bench_dp2_gloo.json 2> gpurun_out/r8z_bench_dp2_gloo.log || { tail -30 gpurun_out/r8z_bench_dp2_gloo.log; exit 1; }
cut -c1-600 gpurun_out/r8z_bench_dp2_gloo.json
