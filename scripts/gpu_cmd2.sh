set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-bfs --no-cpu > gpurun_out/bench_plan.json 2> gpurun_out/bench_plan.err
