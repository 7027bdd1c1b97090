#!/bin/bash
# Round-4 probe (through gpurun): A* per-pop clocks after the fused pop / batched pushes, and the
# worker bitmap-staging policy on C5 / wh10k (default vs forced on / off).
set -o pipefail
mkdir -p gpurun_out
TSW_ASTAR_PROF=1 timeout -k 10 120 python scripts/astar_lat.py --diag --label r4heap > gpurun_out/alat_r4.jsonl 2> gpurun_out/alat_r4.err &&
timeout -k 10 150 python -u scripts/scale_bench.py c5 --cpu-steps 1 > gpurun_out/r4p_c5.jsonl 2> gpurun_out/r4p_c5.log &&
for fb in def 0 1; do
  if [ $fb = def ]; then e=""; else e="TSW_WORKER_FB=$fb"; fi
  env $e timeout -k 10 150 python -u scripts/scale_bench.py wh10k --cpu-steps 1 > gpurun_out/r4p_wh_$fb.jsonl 2> gpurun_out/r4p_wh_$fb.log || exit 1
done
