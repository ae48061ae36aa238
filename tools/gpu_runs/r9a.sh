set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bo_encoder" > gpurun_out/r9a_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r9a_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r9a_pytest.txt | head; exit 1; }
timeout -k 10 300 python -u tools/bench_inference.py --batches 1,16 --iters 60 --modes policy_graph,teacher_graph > gpurun_out/r9a_bench_inference.jsonl 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r9a_bench_inference.jsonl | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r9a_p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 2 --precision fp32 --inference 1 --sl 0 > $GRAFT_REPO_ROOT/gpurun_out/r9a_prof.log 2>&1; rc=$?; cd $GRAFT_REPO_ROOT
[ $rc -eq 0 ] || { tail -5 gpurun_out/r9a_prof.log; exit 1; }
f=$(find /tmp/r9a_p -name '*kernel_stats.csv' | head -1); grep -E "bo_fwd|bo_bwd" "$f" | cut -d, -f1-6
APPLESTAR_DIST_BACKEND=gloo timeout -k 20 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --inference 0 --sl 0 > gpurun_out/r8z_bench_dp2_gloo.json 2> gpurun_out/r8z_bench_dp2_gloo.log || { tail -30 gpurun_out/r8z_bench_dp2_gloo.log; exit 1; }
cut -c1-600 gpurun_out/r8z_bench_dp2_gloo.json
