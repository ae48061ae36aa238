set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lstm" > gpurun_out/lstm_pytest.txt 2>&1 || { tail -30 gpurun_out/lstm_pytest.txt; exit 1; }
tail -2 gpurun_out/lstm_pytest.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/lstm_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lstm_f32_$i.json'));print('fp32', $i, d['ms_per_step'])"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/lstm_bf16_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lstm_bf16_$i.json'));print('bf16', $i, d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/lstm_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --precision fp32 --inference 0 > $GRAFT_REPO_ROOT/gpurun_out/lstm_prof.log 2>&1 || exit 1
