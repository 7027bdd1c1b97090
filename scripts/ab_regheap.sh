#!/bin/bash
# A/B (diagnostic build, TSW_* knobs): register-resident A* heap (TSW_ASTAR_REGHEAP=63 default / 0 =
# LDS array only) and the idle-worker wake gate (TSW_WAKE_GATE=k: 1 in 2^k idle workers rescans at
# once on a publish), interleaved; then the C3 plan-debug counters for the gate.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_reg.txt
CFGS="r63g0:TSW_ASTAR_REGHEAP=63 r0g0:TSW_ASTAR_REGHEAP=0 r63g3:TSW_WAKE_GATE=3 r63g5:TSW_WAKE_GATE=5"
for rep in 1 2; do
  for cfg in $CFGS; do
    tag=${cfg%%:*}; e=${cfg#*:}
    env $e timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/ab_reg_c3_$tag.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/ab_reg_c3_$tag.json') if l.startswith('{')][-1]); k=b['kernel_stats']; print('c3 $tag', b['ms_per_step'], round(k['coop_wait_ms']/3,1))" >> gpurun_out/ab_reg.txt
  done
done
for cfg in $CFGS; do
  tag=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 150 python -u scripts/scale_bench.py wh10k --cpu-steps 1 --diag > gpurun_out/ab_reg_wh_$tag.jsonl 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_reg_wh_$tag.jsonl').read().strip().splitlines()[-1]); print('wh10k $tag', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_reg.txt
done
TSW_WAKE_GATE=3 TSW_PLAN_DEBUG=1 timeout -k 10 100 python -u scripts/scale_bench.py c3 --cpu-steps 1 --diag > gpurun_out/c3_dbg_g3.jsonl 2> gpurun_out/c3_dbg_g3.log
cat gpurun_out/ab_reg.txt
