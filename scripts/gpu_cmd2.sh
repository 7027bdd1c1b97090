set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 scripts/scale_bench.py c3 --cpu-steps 2 > gpurun_out/prof_c3.log 2>&1
