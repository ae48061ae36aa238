set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile.py --graph > gpurun_out/t_host_graph.txt 2> gpurun_out/t_host_graph.err || { tail -20 gpurun_out/t_host_graph.err; exit 1; }
