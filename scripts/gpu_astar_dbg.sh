set -o pipefail
export TMPDIR=/tmp
TSW_ASTAR_PROF=1 timeout -k 10 200 python scripts/astar_bench.py --child gpurun_out/astar_d > gpurun_out/astar_dbg.log 2>&1
