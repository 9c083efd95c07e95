#!/bin/bash
# planner: two workgroups per CU for long multi-row slices; parity + the decode configs
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_m 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/merge3.txt
for rep in 1 2; do
  for cfg in "--n-q 64" "--n-q 64 --heads 4 --kv-heads 4" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "" "--kv-type f16 --kv-len 2048"; do
    echo "### $cfg" >> gpurun_out/merge3.txt
    timeout -k 10 120 $B $cfg >> gpurun_out/merge3.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/merge3.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
