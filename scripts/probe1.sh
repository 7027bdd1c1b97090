set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/plan_probe.py > gpurun_out/probe_default.jsonl 2>gpurun_out/probe.err &&
TSW_PLAN_BLOCK=512 timeout -k 10 200 python scripts/plan_probe.py --diag 450 2000 > gpurun_out/probe_b512.jsonl 2>>gpurun_out/probe.err &&
TSW_PLAN_DEBUG=1 timeout -k 10 200 python scripts/plan_probe.py --diag --reps 1 450 2000 > gpurun_out/probe_dbg.jsonl 2>gpurun_out/probe_dbg.err
