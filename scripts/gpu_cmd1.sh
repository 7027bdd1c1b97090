set -o pipefail
export TMPDIR=/tmp
TSW_PLAN_DEBUG=1 timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-bfs --no-cpu > gpurun_out/dbg.json 2> gpurun_out/dbg.log && \
bash scripts/profile_round.sh r1
