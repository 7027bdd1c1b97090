# Round-end measurement: GPU parity suite, bench + rocprofv3 kernel trace + PMC passes,
# scale instances (c3 full, wh10k 30-step prefix), K3 latency micro-bench.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
bash scripts/profile_round.sh r1 &&
timeout -k 10 300 python -u scripts/scale_bench.py c3 > gpurun_out/scale_c3.jsonl 2> gpurun_out/scale_c3.log &&
timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k.jsonl 2> gpurun_out/scale_wh10k.log &&
timeout -k 10 300 python scripts/astar_bench.py --out gpurun_out/astar_bench.json > gpurun_out/astar_bench.log 2>&1
