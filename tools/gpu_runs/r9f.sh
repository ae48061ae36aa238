set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/inference_casts.py --batch 1 --top 80 > gpurun_out/r9f_inference_casts.txt 2>&1 || { tail -10 gpurun_out/r9f_inference_casts.txt; exit 1; }
head -120 gpurun_out/r9f_inference_casts.txt
