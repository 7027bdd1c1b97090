set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/scale_bench.py c3 > gpurun_out/scale_c3.jsonl 2> gpurun_out/scale_c3.log &&
TSW_ASTAR_SERIAL=1 timeout -k 10 300 python -u scripts/scale_bench.py c3 --cpu-steps 2 > gpurun_out/scale_c3_serial.jsonl 2> gpurun_out/scale_c3_serial.log &&
timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k.jsonl 2> gpurun_out/scale_wh10k.log
