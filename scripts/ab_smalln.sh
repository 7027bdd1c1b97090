#!/bin/bash
# worker waves per CU are capped at block/64 in the plan dispatch; a plan with <= 256
# agents gets block 256 (4 worker waves per CU). A/B on C2 (random-32-32-20, 200 agents, lazy next
# hops so the coop workers run): default block vs TSW_PLAN_BLOCK=1024 (16 worker waves per CU).
set -o pipefail
mkdir -p gpurun_out
for b in 0 1024; do
  TSW_PLAN_BLOCK=$b timeout -k 10 120 python bench.py --diag --config c2_random_32_32_20 --nexthop lazy --steps 5 --warmup 1 \
    --no-cpu --no-bfs > gpurun_out/smalln_$b.json 2> gpurun_out/smalln_$b.err || exit 1
done
