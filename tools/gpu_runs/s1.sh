set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s1_bench_fp32.json 2> gpurun_out/s1_bench_fp32.log || { tail -30 gpurun_out/s1_bench_fp32.log; exit 1; }
cat gpurun_out/s1_bench_fp32.json
timeout -k 10 300 python tools/conv_shapes.py --out gpurun_out/s1_conv_shapes_fp32.txt > /dev/null 2> gpurun_out/s1_conv_shapes.log || { tail -30 gpurun_out/s1_conv_shapes.log; exit 1; }
head -40 gpurun_out/s1_conv_shapes_fp32.txt
timeout -k 10 300 python tools/glue_kernels.py --top 60 > gpurun_out/s1_glue_fp32.txt 2>&1 || { tail -30 gpurun_out/s1_glue_fp32.txt; exit 1; }
grep "no frame" gpurun_out/s1_glue_fp32.txt | head -20
