set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "copy or derived or fused or graph or trainer" > gpurun_out/copy3_pytest.txt 2>&1 || { tail -40 gpurun_out/copy3_pytest.txt; exit 1; }
tail -1 gpurun_out/copy3_pytest.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/copy3_f32_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/copy3_f32_$i.json'));print('fp32', $i, d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/copy3_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --precision fp32 --inference 0 > $GRAFT_REPO_ROOT/gpurun_out/copy3_prof.log 2>&1 || exit 1
