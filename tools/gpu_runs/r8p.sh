set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/sync_audit.py --precision fp32 > gpurun_out/r8p_sync_fp32.txt 2>&1 || { tail -20 gpurun_out/r8p_sync_fp32.txt; exit 1; }
head -40 gpurun_out/r8p_sync_fp32.txt
timeout -k 10 300 python -u tools/sync_audit.py --precision bf16 > gpurun_out/r8p_sync_bf16.txt 2>&1 || { tail -20 gpurun_out/r8p_sync_bf16.txt; exit 1; }
head -40 gpurun_out/r8p_sync_bf16.txt
