set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
for b in 64 128 256; do
  TSW_PLAN_DEBUG=1 TSW_PLAN_BLOCK=$b timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-bfs --no-cpu > gpurun_out/blk$b.json 2> gpurun_out/blk$b.log || exit 1
done
