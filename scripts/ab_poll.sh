#!/bin/bash
# A/B (diagnostic build): idle-worker polling — wake gate (TSW_WAKE_GATE) and slow pollers
# (TSW_SLOW_POLL=k: only 1 in 2^k idle workers polls at full rate, the others TSW_SLOW_MULT times
# slower), C3 plans interleaved, then wh10k / C5 once each and the C3 queue-delay counters.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab_poll.txt
CFGS="base:TSW_WAKE_GATE=0 f4m64g2:TSW_SLOW_POLL=4,TSW_SLOW_MULT=64,TSW_WAKE_GATE=2 f5m64g1:TSW_SLOW_POLL=5,TSW_SLOW_MULT=64,TSW_WAKE_GATE=1 f4m256g2:TSW_SLOW_POLL=4,TSW_SLOW_MULT=256,TSW_WAKE_GATE=2 f6m64g0:TSW_SLOW_POLL=6,TSW_SLOW_MULT=64"
for rep in 1 2; do
  for cfg in $CFGS; do
    tag=${cfg%%:*}; e=${cfg#*:}; e=${e//,/ }
    env $e timeout -k 10 200 python bench.py --diag --steps 3 --warmup 1 --no-cpu --no-bfs --no-sharded > gpurun_out/ab_poll_c3_$tag.json 2>/dev/null || exit 1
    python -c "import json; b=json.loads([l for l in open('gpurun_out/ab_poll_c3_$tag.json') if l.startswith('{')][-1]); k=b['kernel_stats']; print('c3 $tag', b['ms_per_step'], round(k['coop_wait_ms']/3,1))" >> gpurun_out/ab_poll.txt
  done
done
for cfg in $CFGS; do
  tag=${cfg%%:*}; e=${cfg#*:}; e=${e//,/ }
  for inst in wh10k c5; do
    env $e timeout -k 10 150 python -u scripts/scale_bench.py $inst --cpu-steps 1 --diag > gpurun_out/ab_poll_${inst}_$tag.jsonl 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/ab_poll_${inst}_$tag.jsonl').read().strip().splitlines()[-1]); print('$inst $tag', d['gpu_end_to_end_s'], d['coop_wait_ms'], d['prefix_bit_exact'])" >> gpurun_out/ab_poll.txt
  done
done
for cfg in $CFGS; do
  tag=${cfg%%:*}; e=${cfg#*:}; e=${e//,/ }
  env $e TSW_PLAN_DEBUG=1 timeout -k 10 100 python -u scripts/scale_bench.py c3 --cpu-steps 1 --diag > /dev/null 2> gpurun_out/ab_poll_dbg_$tag.log || exit 1
  echo "$tag $(grep 'queue delay' gpurun_out/ab_poll_dbg_$tag.log | tail -1)" >> gpurun_out/ab_poll.txt
done
cat gpurun_out/ab_poll.txt
grep -h "detour staging" gpurun_out/ab_poll_dbg_*.log >> gpurun_out/ab_poll.txt; tail -5 gpurun_out/ab_poll.txt
