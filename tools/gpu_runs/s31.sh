set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/glue_kernels.py --top 45 --shapes --match CUDAFunctor_add,Fill,copy,threshold > gpurun_out/s31_glue_shapes.txt 2>&1 || { tail -20 gpurun_out/s31_glue_shapes.txt; exit 1; }
grep -v "amdgpu\|Warning\|warn" gpurun_out/s31_glue_shapes.txt | head -50
