#!/bin/bash
# second-launch merge for multi-row split tiles: parity, then A/B against the fused last-arriver merge
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_m 900 python -u -m pytest tests -m gpu -q --maxfail 20 -p no:cacheprovider --timeout 180 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/merge.txt
for rep in 1; do
  for cfg in "--n-q 64 --heads 4 --kv-heads 4" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "--n-q 64" ""; do
    for v in "" "--fused-merge"; do
      echo "### $cfg $v" >> gpurun_out/merge.txt
      timeout -k 10 120 $B $cfg $v >> gpurun_out/merge.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/merge.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
