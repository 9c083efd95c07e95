#!/bin/bash
# phase costs of the multi-row (config 5 shard) and one-row (config 3) decode: full vs diagnostic builds
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/diag5.txt
for rep in 1 2; do
  for cfg in "--n-q 64 --heads 4 --kv-heads 4" "" "--kv-type q4_0 --kv-heads 8 --kv-len 8192"; do
    for lib in libfattn.so libfattn_diag_noatomic.so libfattn_diag_nopublish.so libfattn_diag_notail.so libfattn_diag_dmaonly.so; do
      echo "### $cfg $lib" >> gpurun_out/diag5.txt
      FATTN_LIB=$lib timeout -k 10 120 $B $cfg >> gpurun_out/diag5.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/diag5.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
