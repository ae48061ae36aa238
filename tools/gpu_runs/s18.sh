set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision fp32 > gpurun_out/s18_timeline_fp32.txt 2>&1 || { tail -20 gpurun_out/s18_timeline_fp32.txt; exit 1; }
grep -v amdgpu gpurun_out/s18_timeline_fp32.txt | tail -60
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision bf16 > gpurun_out/s18_timeline_bf16.txt 2>&1 || { tail -20 gpurun_out/s18_timeline_bf16.txt; exit 1; }
grep -v amdgpu gpurun_out/s18_timeline_bf16.txt | tail -20
