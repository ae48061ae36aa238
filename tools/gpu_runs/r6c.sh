set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in fp32 bf16; do
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/r6c_$P -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 --precision $P --inference 0 > /tmp/r6c_$P.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 /tmp/r6c_$P.log; exit 1; }
python tools/prof_steady.py $(find /tmp/r6c_$P -name '*kernel_trace.csv' | head -1) 3 70 > gpurun_out/r6c_steady_$P.txt && head -12 gpurun_out/r6c_steady_$P.txt
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/r6c_bench_bf16.json 2> gpurun_out/r6c_bench_bf16.log || exit 1
python -c "import json;d=json.load(open('gpurun_out/r6c_bench_bf16.json'));print('bf16', d['ms_per_step'])"
