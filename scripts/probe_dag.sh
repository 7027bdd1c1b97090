# DAG early-exit A/B on the C3 plan (diagnostic library, planner debug counters) -> gpurun_out/dag_*.jsonl/.err
# usage: bash scripts/probe_dag.sh "ENV=.." ... (one plan_probe per setting)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
export TSW_PLAN_DEBUG=1
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python scripts/plan_probe.py --diag --reps 2 2000 > gpurun_out/dag_$i.jsonl 2> gpurun_out/dag_$i.err || exit $?
  i=$((i+1))
done
