# C2 k_plan sub-phase ticks (TSW_PLAN_DEBUG) with the eager (default) policy.
set -o pipefail
export TMPDIR=/tmp
TSW_PLAN_DEBUG=1 timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-bfs > gpurun_out/c2_dbg.json 2> gpurun_out/c2_dbg.err
