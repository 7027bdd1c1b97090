#!/bin/bash
# wh10k planner probe (run through gpurun): the AG-false parity tests, then a 200-step wh10k plan
# with k_plan sub-phase ticks, with the default placement and with TSW_PLAN_AP=0 (A/B).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "global_agent" --timeout 300 \
  --timeout-method thread > gpurun_out/ap_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
TSW_PLAN_DEBUG=1 timeout -k 10 300 python -u scripts/scale_bench.py wh10k --max-t ${1:-200} > gpurun_out/wh_dbg.jsonl 2> gpurun_out/wh_dbg.log &&
TSW_PLAN_AP=0 TSW_PLAN_DEBUG=1 timeout -k 10 300 python -u scripts/scale_bench.py wh10k --max-t ${1:-200} > gpurun_out/wh_dbg0.jsonl 2> gpurun_out/wh_dbg0.log
