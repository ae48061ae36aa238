set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/glue_kernels.py --precision fp32 --top 60 > gpurun_out/r9k_glue_fp32.txt 2>&1 || { tail -20 gpurun_out/r9k_glue_fp32.txt; exit 1; }
grep -v "amdgpu.ids\|Warning\|warn" gpurun_out/r9k_glue_fp32.txt | head -70
