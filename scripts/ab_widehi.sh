#!/bin/bash
# A/B (diagnostic build): walk-ahead depth on small grids (TSW_WIDE_HI, default 16) on wh10k and C3.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_widehi.txt
for h in 16 32 24 12; do
  TSW_WIDE_HI=$h timeout -k 10 200 python -u scripts/scale_bench.py wh10k --cpu-steps 1 --diag > gpurun_out/abw.jsonl 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abw.jsonl').read().strip().splitlines()[-1]); print('wh10k hi=$h', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_widehi.txt
  TSW_WIDE_HI=$h timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/abw.json 2>/dev/null || exit 1
  python -c "import json; b=json.loads([l for l in open('gpurun_out/abw.json') if l.startswith('{')][-1]); print('c3 hi=$h', b['ms_per_step'], round(b['kernel_stats']['coop_wait_ms']/3,1))" >> gpurun_out/ab_widehi.txt
done
cat gpurun_out/ab_widehi.txt
