set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/host_profile.py --precision fp32 --steps 8 --top 60 > gpurun_out/r8l_host_profile_fp32.txt 2>&1 || { tail -5 gpurun_out/r8l_host_profile_fp32.txt; exit 1; }
head -100 gpurun_out/r8l_host_profile_fp32.txt
