set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/astar_lat.py > gpurun_out/alat2.jsonl 2>gpurun_out/alat.err &&
timeout -k 10 200 python scripts/plan_probe.py 450 2000 > gpurun_out/probe_label.jsonl 2>gpurun_out/probe.err &&
for i in 1 2 3; do TSW_PLAN_DEBUG=1 timeout -k 10 200 python -u scripts/scale_bench.py wh10k --cpu-steps 1 --diag >> gpurun_out/wh10k_dbg.jsonl 2>> gpurun_out/wh10k_dbg.err || exit 1; done &&
timeout -k 10 900 python -u scripts/scale_bench.py wh10k --cpu-steps 100 --cpu-windows 20 > gpurun_out/wh10k_cpu100.jsonl 2> gpurun_out/wh10k_cpu100.err
