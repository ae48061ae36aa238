set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision fp32 > gpurun_out/r8q_timeline_fp32.txt 2>&1 || { tail -20 gpurun_out/r8q_timeline_fp32.txt; exit 1; }
cat gpurun_out/r8q_timeline_fp32.txt
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision bf16 > gpurun_out/r8q_timeline_bf16.txt 2>&1 || { tail -20 gpurun_out/r8q_timeline_bf16.txt; exit 1; }
cat gpurun_out/r8q_timeline_bf16.txt
