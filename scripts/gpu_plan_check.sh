set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
TSW_PLAN_DEBUG=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-bfs --no-cpu > gpurun_out/plan_dbg.json 2> gpurun_out/plan_dbg.log &&
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-bfs --no-cpu > gpurun_out/plan_bench.json 2> gpurun_out/plan_bench.log
