# C2 headline A/B: eager vs lazy next-hop policy, plus k_plan sub-phase ticks (TSW_PLAN_DEBUG).
set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-bfs"
timeout -k 10 120 $B --nexthop eager > gpurun_out/c2_eager.json 2> gpurun_out/c2_eager.err &&
timeout -k 10 120 $B --nexthop lazy > gpurun_out/c2_lazy.json 2> gpurun_out/c2_lazy.err &&
TSW_PLAN_DEBUG=1 timeout -k 10 120 $B --nexthop eager > gpurun_out/c2_dbg.json 2> gpurun_out/c2_dbg.err
