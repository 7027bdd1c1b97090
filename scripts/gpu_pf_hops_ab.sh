# A/B: wide-prefetch horizon (TSW_WIDE_PREFETCH hops) on c3 and the wh10k prefix.
set -o pipefail
export TMPDIR=/tmp
for h in ${HOPS:-8 16}; do
TSW_WIDE_PREFETCH=$h timeout -k 10 300 python -u scripts/scale_bench.py c3 > gpurun_out/scale_c3_h$h.jsonl 2> gpurun_out/scale_c3_h$h.log &&
TSW_WIDE_PREFETCH=$h timeout -k 10 400 python -u scripts/scale_bench.py wh10k --max-t 30 > gpurun_out/scale_wh10k_h$h.jsonl 2> gpurun_out/scale_wh10k_h$h.log || exit 1
done
