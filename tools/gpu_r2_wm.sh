#!/bin/bash
# one-row tiles: fused workgroup-row merge (default) vs LDS merge + second-launch merge (--wave-merge 1)
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/wm.txt
for rep in 1 2; do
  for cfg in "" "--kv-type f16 --kv-len 2048" "--kv-len 32768 --heads 8 --kv-heads 8" "--waves 4"; do
    for v in "" "--wave-merge 1"; do
      echo "### $cfg $v" >> gpurun_out/wm.txt
      timeout -k 10 120 $B $cfg $v >> gpurun_out/wm.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/wm.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
