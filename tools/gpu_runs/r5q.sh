set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/debug_gated_bf16.py > gpurun_out/r5q_debug_gated.txt 2>&1; echo "debug rc=$?"; cat gpurun_out/r5q_debug_gated.txt | grep -v amdgpu.ids
for v in both nogemm noconv none both2; do
  case $v in both|both2) E="";; nogemm) E="APPLESTAR_GEMM_PSB=0";; noconv) E="APPLESTAR_CONV_PSB=0";; none) E="APPLESTAR_GEMM_PSB=0 APPLESTAR_CONV_PSB=0";; esac
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 5 --precision fp32 --inference 0 > gpurun_out/r5q_bench_$v.json 2> gpurun_out/r5q_bench_$v.log || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r5q_bench_$v.json'));print('$v', d['ms_per_step'])"
done
# learner step time while another process serves inference graphs flat out on the same GPU
timeout -k 10 200 python -u tools/bench_inference.py --batches 16 --iters 3000 --modes policy_graph > gpurun_out/r5q_bg_inference.log 2>&1 &
BG=$!
sleep 25
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --precision fp32 --inference 0 > gpurun_out/r5q_bench_coinference.json 2> gpurun_out/r5q_bench_coinference.log; rc=$?
kill $BG 2>/dev/null; wait $BG 2>/dev/null
python -c "import json;d=json.load(open('gpurun_out/r5q_bench_coinference.json'));print('with concurrent inference', d['ms_per_step'])"
[ $rc -eq 0 ] || exit 1
