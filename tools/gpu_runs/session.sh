set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "copy or mixed or master or trainer or two_ranks" > gpurun_out/cv_pytest.txt 2>&1 || { tail -40 gpurun_out/cv_pytest.txt; exit 1; }
tail -1 gpurun_out/cv_pytest.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/cv_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --precision bf16 --inference 0 > $GRAFT_REPO_ROOT/gpurun_out/cv_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --precision bf16 --inference 0 > gpurun_out/cv_bf16_$i.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/cv_bf16_$i.json'));print('bf16', $i, d['ms_per_step'])"
done
