# A/B: k_astar_wave LDS heap capacity (more waves per CU vs heap overflows), wh10k prefix.
set -o pipefail
export TMPDIR=/tmp
TSW_ASTAR_WAVE_HCAP=2048 timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k_h2048.jsonl 2> gpurun_out/scale_wh10k_h2048.log &&
TSW_ASTAR_WAVE_HCAP=1024 timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k_h1024.jsonl 2> gpurun_out/scale_wh10k_h1024.log
