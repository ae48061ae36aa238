set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/s36_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/s36_pytest.txt; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
  for v in base old; do
    case $v in base) E="";; old) E="APPLESTAR_COLRED_V4_MIN=-1";; esac
    env $E timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/s36_fp32_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/s36_fp32_${v}_$i.json'));print('fp32 $v', $i, d['ms_per_step'])"
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p36a -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 --precision fp32 --inference 0 > $R/gpurun_out/s36_prof_a.log 2>&1 || { tail -20 $R/gpurun_out/s36_prof_a.log; exit 1; }
export APPLESTAR_COLRED_V4_MIN=-1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p36b -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 3 --precision fp32 --inference 0 > $R/gpurun_out/s36_prof_b.log 2>&1 || { tail -20 $R/gpurun_out/s36_prof_b.log; exit 1; }
cd $R
ta=$(find /tmp/p36a -name '*kernel_trace.csv' | head -1); tb=$(find /tmp/p36b -name '*kernel_trace.csv' | head -1)
python3 tools/prof_steady.py "$ta" 3 80 > gpurun_out/s36_steady_v4.txt
python3 tools/prof_steady.py "$tb" 3 80 > gpurun_out/s36_steady_old.txt
grep -h "column_reduce\|kernels / iteration" gpurun_out/s36_steady_v4.txt gpurun_out/s36_steady_old.txt | cut -c1-140
