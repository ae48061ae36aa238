set -o pipefail
mkdir -p gpurun_out
APPLESTAR_LSTM_FWD_GRANULE=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "lstm" > gpurun_out/r6i_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r6i_pytest.txt; [ $rc -eq 0 ] || exit 1
b() {  # name precision env...
  N=$1; P=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision $P --inference 0 > gpurun_out/r6i_bench_$N.json 2> gpurun_out/r6i_bench_$N.log || { tail -5 gpurun_out/r6i_bench_$N.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6i_bench_$N.json'));print('$N', d['ms_per_step'])"
}
b fp32_gran fp32 APPLESTAR_LSTM_FWD_GRANULE=1 || exit 1
b fp32_flag fp32 APPLESTAR_LSTM_FWD_GRANULE=0 || exit 1
b bf16_gran bf16 APPLESTAR_LSTM_FWD_GRANULE=1 || exit 1
b bf16_flag bf16 APPLESTAR_LSTM_FWD_GRANULE=0 || exit 1
cd /tmp && APPLESTAR_LSTM_FWD_GRANULE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6i_prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --precision fp32 --inference 0 > /tmp/r6i_prof.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || exit 1
grep -h "lnlstm" $(find /tmp/r6i_prof -name '*kernel_stats.csv' | head -1) | cut -c1-200
