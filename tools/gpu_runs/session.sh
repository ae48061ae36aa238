set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/glue_sites.py --steps 1 --shapes > gpurun_out/glue_sites_fp32_shapes.txt 2> gpurun_out/glue_sites.err || { tail -20 gpurun_out/glue_sites.err; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "copy" > gpurun_out/copy_pytest.txt 2>&1 || { tail -30 gpurun_out/copy_pytest.txt; exit 1; }
tail -2 gpurun_out/copy_pytest.txt
