#!/bin/bash
# decode A/B on config 3 (and 2, 4): loader-wave kernel variants vs the split kernel
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
C2="--kv-type f16 --kv-len 2048"
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
for rep in 1 2; do
for cfg in "" "$C4"; do
  for v in "--dec 1" "--dec 2 --dec-compute 8 --dec-loaders 1 --dec-ahead 3" "--dec 2 --dec-compute 8 --dec-loaders 1 --dec-ahead 5" \
           "--dec 2 --dec-compute 8 --dec-loaders 2 --dec-ahead 2" "--dec 2 --dec-compute 8 --dec-loaders 2 --dec-ahead 3" \
           "--dec 2 --dec-compute 4 --dec-loaders 1 --dec-ahead 4" "--dec 2 --dec-compute 8 --dec-loaders 1 --dec-ahead 4 --wave-merge 1" \
           "--dec 2 --dec-compute 4 --dec-loaders 1 --dec-ahead 4 --wave-merge 1"; do
    echo "### $cfg $v" >> gpurun_out/ab.txt
    timeout -k 10 120 $B $cfg $v >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
done
grep -E "###|kernel_ms_avg" gpurun_out/ab.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*/  kernel_ms \1 median \2 frac \3/'
