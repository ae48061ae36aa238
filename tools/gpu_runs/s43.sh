set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p43 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 --precision fp32 --inference 0 > $R/gpurun_out/s43_prof.log 2>&1 || { tail -20 $R/gpurun_out/s43_prof.log; exit 1; }
cd $R
t=$(find /tmp/p43 -name '*kernel_trace.csv' | head -1)
python3 tools/prof_steady.py "$t" 3 80 > gpurun_out/s43_steady_fp32.txt
head -9 gpurun_out/s43_steady_fp32.txt
timeout -k 10 300 python tools/glue_kernels.py --top 40 --shapes --match CUDAFunctor_add,Fill,copy,threshold > gpurun_out/s43_glue_shapes.txt 2>&1 || { tail -5 gpurun_out/s43_glue_shapes.txt; exit 1; }
grep -v Warning gpurun_out/s43_glue_shapes.txt | grep "ms " | head -12 | cut -c1-160
