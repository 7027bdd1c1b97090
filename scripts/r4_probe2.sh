#!/bin/bash
# Round-4 probe 2: register-resident A* heap — GPU parity, A* per-pop clocks, C3 / C5 / wh10k plans.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_run.sh tests &&
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -q " failed" gpurun_out/gpu_tests.log &&
TSW_ASTAR_PROF=1 timeout -k 10 120 python scripts/astar_lat.py --diag --label r4reg > gpurun_out/alat_r4b.jsonl 2> gpurun_out/alat_r4b.err &&
bash scripts/gpu_run.sh plan &&
timeout -k 10 150 python -u scripts/scale_bench.py c5 --cpu-steps 1 > gpurun_out/r4q_c5.jsonl 2> gpurun_out/r4q_c5.log &&
timeout -k 10 150 python -u scripts/scale_bench.py wh10k --cpu-steps 1 > gpurun_out/r4q_wh.jsonl 2> gpurun_out/r4q_wh.log
