set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "entity or parity" > gpurun_out/ent3_pytest.txt 2>&1 || { tail -40 gpurun_out/ent3_pytest.txt; exit 1; }
tail -1 gpurun_out/ent3_pytest.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/ent3_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --precision fp32 --inference 0 > $GRAFT_REPO_ROOT/gpurun_out/ent3_prof.log 2>&1 || exit 1
