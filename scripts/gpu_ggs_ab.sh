# A/B: k_astar_wave first tier with g_scores in LDS (default) vs global slots (TSW_ASTAR_GLOBAL_GS=1), wh10k prefix.
set -o pipefail
export TMPDIR=/tmp
TSW_ASTAR_GLOBAL_GS=1 timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k_ggs.jsonl 2> gpurun_out/scale_wh10k_ggs.log &&
TSW_ASTAR_GLOBAL_GS=1 timeout -k 10 300 python -u scripts/scale_bench.py c3 > gpurun_out/scale_c3_ggs.jsonl 2> gpurun_out/scale_c3_ggs.log
