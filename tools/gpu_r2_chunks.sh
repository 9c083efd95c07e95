#!/bin/bash
# chunk-length sweep for the multi-row configs now that their merge is a second launch
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/chunks.txt
for cfg in "--n-q 64 --heads 4 --kv-heads 4" "--n-q 64" "--kv-type q4_0 --kv-heads 8 --kv-len 8192"; do
  for ch in 0 128 256 512 1024; do
    for w in 0 8; do
      echo "### $cfg --kv-chunk $ch --waves $w" >> gpurun_out/chunks.txt
      timeout -k 10 120 $B $cfg --kv-chunk $ch --waves $w >> gpurun_out/chunks.txt 2>&1 || echo "rc=$?" >> gpurun_out/chunks.txt
    done
  done
done
grep -E "###|kernel_ms_avg|rc=" gpurun_out/chunks.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
