#!/bin/bash
# A/B of planner knobs on a scale instance (run through gpurun from the repo root).
# Usage: bash scripts/ab_scale.sh INSTANCE MAX_T "ENV1=a ENV2=b" "ENV1=c" ...  (TSW_PLAN_DEBUG on)
#   -> gpurun_out/abs_<i>.jsonl / .log
set -o pipefail
mkdir -p gpurun_out
inst=$1; mt=$2; shift 2
i=0
for e in "$@"; do
  echo "[abs] $i: $e"
  env $e TSW_PLAN_DEBUG=1 timeout -k 10 300 python -u scripts/scale_bench.py $inst --max-t $mt --cpu-steps 1 --diag \
    > gpurun_out/abs_$i.jsonl 2> gpurun_out/abs_$i.log || exit $?
  i=$((i+1))
done
