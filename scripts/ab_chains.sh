#!/bin/bash
# A/B (diagnostic build): task-chain workers on / off (TSW_TASK_CHAINS) on C3, interleaved.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_chains.txt
for rep in 1 2; do
  for c in 1 0; do
    TSW_TASK_CHAINS=$c timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/abc.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abc.json') if l.startswith('{')][-1]); print('c3 chains=$c', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_chains.txt
  done
done
cat gpurun_out/ab_chains.txt
