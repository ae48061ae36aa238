#!/bin/bash
# First MI355X pass: GPU tests, torch-only vs native bench, rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch; print(torch.__version__, torch.cuda.get_device_name(0))" > gpurun_out/env.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-native > gpurun_out/bench_torch.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_native.log 2>&1 || exit 1
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "prof exit $?"
