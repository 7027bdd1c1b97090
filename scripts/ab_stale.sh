#!/bin/bash
# A/B of the coop workers' stale-speculation drop (TSW_SPEC_STALE = steps, 0 = off), diagnostic build:
# C5 with the planner's debug counters, then C3 + wh10k full horizon. Each run has its own limit.
set -o pipefail
mkdir -p gpurun_out
for s in ${STALE_LIST:-16 0 4 64}; do
  TSW_SPEC_STALE=$s TSW_PLAN_DEBUG=1 timeout -k 10 150 python -u scripts/scale_bench.py c5 --cpu-steps 1 --diag \
    > gpurun_out/c5s_$s.jsonl 2> gpurun_out/c5s_$s.log || exit 1
done
for s in ${STALE_LIST2:-16 0}; do
  TSW_SPEC_STALE=$s timeout -k 10 200 python -u scripts/scale_bench.py c3 wh10k --cpu-steps 1 --diag \
    > gpurun_out/c3s_$s.jsonl 2> gpurun_out/c3s_$s.log || exit 1
done
