set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in fp32 bf16; do
timeout -k 10 300 python -u tools/host_gpu_timeline.py --precision $P > gpurun_out/r9c_timeline_$P.txt 2>&1 || { tail -20 gpurun_out/r9c_timeline_$P.txt; exit 1; }
grep -v amdgpu gpurun_out/r9c_timeline_$P.txt
done
