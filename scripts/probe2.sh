set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/astar_lat.py > gpurun_out/alat.jsonl 2>gpurun_out/alat.err &&
TSW_ASTAR_OLDPOP=1 timeout -k 10 120 python scripts/astar_lat.py --diag --label oldpop >> gpurun_out/alat.jsonl 2>>gpurun_out/alat.err &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "astar or golden or parity or c3_full" > gpurun_out/t_astar.log 2>&1 &&
timeout -k 10 200 python scripts/plan_probe.py 450 2000 > gpurun_out/probe_pop.jsonl 2>gpurun_out/probe.err
