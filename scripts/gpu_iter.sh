# Iteration check: GPU parity suite, C2 bench, C3 and wh10k (31-step prefix) scale instances.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-bfs > gpurun_out/c2_dbg.json 2> gpurun_out/c2_dbg.err &&
timeout -k 10 300 python -u scripts/scale_bench.py c3 > gpurun_out/scale_c3.jsonl 2> gpurun_out/scale_c3.log &&
timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k.jsonl 2> gpurun_out/scale_wh10k.log
