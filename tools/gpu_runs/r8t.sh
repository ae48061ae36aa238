set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "su_sample" > gpurun_out/r8t_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r8t_pytest.txt; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/r8t_pytest.txt | head; exit 1; }
timeout -k 10 200 python -u tools/bench_su_sample.py > gpurun_out/r8t_su.jsonl 2>&1 || { tail -5 gpurun_out/r8t_su.jsonl; exit 1; }
grep -v amdgpu.ids gpurun_out/r8t_su.jsonl
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU -d /tmp/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_su_sample.py 2 > $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc1.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc1.log; exit 1; }
f=$(find /tmp/p1 -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/tools/pmc_table.py "$f" su_sample > $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc1.txt; head -80 $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc1.txt
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d /tmp/p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_su_sample.py 2 > $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc2.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc2.log; exit 1; }
f=$(find /tmp/p2 -name '*counter_collection.csv' | head -1); python3 $GRAFT_REPO_ROOT/tools/pmc_table.py "$f" su_sample > $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc2.txt; head -80 $GRAFT_REPO_ROOT/gpurun_out/r8t_pmc2.txt
