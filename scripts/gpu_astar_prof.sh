set -o pipefail
export TMPDIR=/tmp
cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/astar_prof -o astar -- python3 scripts/astar_bench.py --child gpurun_out/astar_p > gpurun_out/astar_prof.log 2>&1
