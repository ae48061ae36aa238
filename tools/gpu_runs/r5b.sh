set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/learn_curves.py --out gpurun_out/r5b_learn_curves.json > gpurun_out/r5b_learn.log 2>&1 || { tail -20 gpurun_out/r5b_learn.log; exit 1; }
grep run gpurun_out/r5b_learn.log | cut -c1-900
timeout -k 10 300 python tools/glue_sites.py --steps 2 --precision fp32 --shapes > gpurun_out/r5b_glue_sites_fp32.txt 2>&1 || { tail gpurun_out/r5b_glue_sites_fp32.txt; exit 1; }
head -3 gpurun_out/r5b_glue_sites_fp32.txt
TAG=r5b_fp32 ITERS=5 STEADY=3 BENCH_ARGS="--precision fp32 --steps 3 --warmup 2 --inference 0" bash tools/gpu_prof.sh
