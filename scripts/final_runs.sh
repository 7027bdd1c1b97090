#!/bin/bash
# Round-end runs at the final build (through gpurun, repo root): smoke(), the driver's default bench line
# (profiled traffic paired by build id), pytest -m gpu, full-horizon scale runs with CPU-oracle prefixes,
# per-context HBM, in-dispatch pop cost, lone-query A* latency. Each GPU step has its own time limit.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench_driver_style.json 2> $O/bench_driver_style.err &&
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/scale_bench.py c3 --cpu-steps 101 > $O/scale_c3.jsonl 2> $O/scale_c3.err &&
timeout -k 10 200 python -u scripts/scale_bench.py wh10k --cpu-steps 11 > $O/scale_wh10k.jsonl 2> $O/scale_wh10k.err &&
timeout -k 10 200 python -u scripts/scale_bench.py c5 --cpu-steps 11 > $O/scale_c5.jsonl 2> $O/scale_c5.err &&
timeout -k 10 300 python -u scripts/ctx_hbm.py > $O/ctx_hbm.jsonl 2> $O/ctx_hbm.err &&
timeout -k 10 300 python -u scripts/pop_cost.py c3 wh10k c5 > $O/pop_cost.jsonl 2> $O/pop_cost.err &&
timeout -k 10 200 python -u scripts/astar_lat.py > $O/astar_latency.txt 2> $O/astar_latency.err
