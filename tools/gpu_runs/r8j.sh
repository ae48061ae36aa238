set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r8j_fp32 ITERS=6 STEADY=3 BENCH_ARGS="--precision fp32 --steps 3 --warmup 3 --inference 0 --sl 0" bash tools/gpu_prof.sh || exit 1
timeout -k 10 300 python -u tools/glue_sites.py --steps 2 --precision fp32 --premask > gpurun_out/r8j_glue_premask.txt 2>&1 || { tail -5 gpurun_out/r8j_glue_premask.txt; exit 1; }
head -60 gpurun_out/r8j_glue_premask.txt
