# fp32 steady-state profile
O=gpurun_out/r3f; mkdir -p $O
TAG=r3f_fp32 ITERS=7 STEADY=3 PROF_TIMEOUT=500 BENCH_ARGS="--precision fp32 --steps 4 --warmup 3 --inference 0" timeout -k 10 560 bash tools/gpu_prof.sh > $O/prof_fp32.out 2>&1
