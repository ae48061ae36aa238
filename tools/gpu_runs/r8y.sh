set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in fp32 bf16; do
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision $P > gpurun_out/r8y_timeline_$P.txt 2>&1 || { tail -20 gpurun_out/r8y_timeline_$P.txt; exit 1; }
APPLESTAR_ABL_NO_WGRAD=1 timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision $P > gpurun_out/r8y_timeline_${P}_nowgrad.txt 2>&1 || { tail -20 gpurun_out/r8y_timeline_${P}_nowgrad.txt; exit 1; }
grep -E "host_ms|backward|loss>|fwd:core_lstm<" gpurun_out/r8y_timeline_$P.txt gpurun_out/r8y_timeline_${P}_nowgrad.txt
done
