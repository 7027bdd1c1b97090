#!/bin/bash
# A/B of planner knobs on the bench's planning leg (run through gpurun from the repo root).
# Usage: bash scripts/ab_plan.sh "ENV1=a ENV2=b" "ENV1=c" ...  (one bench planning run per setting,
# TSW_PLAN_DEBUG on) -> gpurun_out/ab_<i>.json / .err
set -o pipefail
mkdir -p gpurun_out
i=0
for e in "$@"; do
  echo "[ab] $i: $e"
  env $e TSW_PLAN_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --no-bfs \
    > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit $?
  i=$((i+1))
done
