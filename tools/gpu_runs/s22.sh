set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/host_profile.py --precision bf16 --steps 10 --top 45 > gpurun_out/s22_host_profile_bf16.txt 2>&1 || { tail -20 gpurun_out/s22_host_profile_bf16.txt; exit 1; }
grep -v amdgpu gpurun_out/s22_host_profile_bf16.txt | head -120
