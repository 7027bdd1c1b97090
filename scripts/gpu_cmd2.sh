set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_10k -o run -- python3 scripts/scale_bench.py wh10k --max-t 30 --cpu-steps 1 > gpurun_out/prof_10k.log 2>&1
