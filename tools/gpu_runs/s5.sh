set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  for r in 32 48 24; do
    APPLESTAR_WGRAD_SMALL_R=$r timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s5_fp32_sr${r}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s5_fp32_sr${r}_$i.json'));print('fp32 small_r=$r', $i, d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/p5 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 --precision fp32 --inference 0 > $R/gpurun_out/s5_prof.log 2>&1 || { tail -20 $R/gpurun_out/s5_prof.log; exit 1; }
cd $R
t=$(find /tmp/p5 -name '*kernel_trace.csv' | head -1)
python3 tools/prof_steady.py "$t" 3 70 > gpurun_out/s5_steady_fp32.txt
head -12 gpurun_out/s5_steady_fp32.txt
