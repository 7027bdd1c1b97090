#!/bin/bash
# A/B (diagnostic build): share of workers walking task chains (TSW_CHAIN_MASK: (wid & m) == m) on
# wh10k and C5 (default 3: a quarter) and C3 (default 1: a half).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_chainmask.txt
for inst in wh10k c5; do
  for m in 3 1 0 7; do
    TSW_CHAIN_MASK=$m timeout -k 10 200 python -u scripts/scale_bench.py $inst --cpu-steps 1 --diag > gpurun_out/abm.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abm.jsonl').read().strip().splitlines()[-1]); print('$inst mask=$m', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_chainmask.txt
  done
done
for m in 1 0 3; do
  TSW_CHAIN_MASK=$m timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/abm.json 2>/dev/null || exit 1
  python -c "import json; b=json.loads([l for l in open('gpurun_out/abm.json') if l.startswith('{')][-1]); print('c3 mask=$m', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_chainmask.txt
done
cat gpurun_out/ab_chainmask.txt
