#!/bin/bash
# A/B (diagnostic build): DAG levels queued past the walk-ahead's first unresolved cell (TSW_DAG_PREFETCH,
# default 6), C3 interleaved x3, wh10k and C5 once each.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_dagpf.txt
for rep in 1 2 3; do
  for d in 6 3; do
    TSW_DAG_PREFETCH=$d timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/abd2.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/abd2.json') if l.startswith('{')][-1]); print('c3 dag=$d', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_dagpf.txt
  done
done
for inst in wh10k c5; do
  for d in 6 3; do
    TSW_DAG_PREFETCH=$d timeout -k 10 200 python -u scripts/scale_bench.py $inst --cpu-steps 1 --diag > gpurun_out/abd2.jsonl 2>/dev/null || exit 1
    python -c "import json; x=json.loads(open('gpurun_out/abd2.jsonl').read().strip().splitlines()[-1]); print('$inst dag=$d', x['gpu_end_to_end_s'], x['coop_wait_ms'], x['prefix_bit_exact'])" >> gpurun_out/ab_dagpf.txt
  done
done
cat gpurun_out/ab_dagpf.txt
