#!/bin/bash
# phase decomposition of the split kernel from diagnostic libraries (tools/build_diag.sh)
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/diag.txt
for cfg in "--waves 16" "--waves 4" "--kv-type f16 --kv-len 2048" "--kv-type q4_0 --kv-heads 8 --kv-len 8192"; do
  for lib in libfattn.so libfattn_diag_notail.so libfattn_diag_nopublish.so libfattn_diag_noatomic.so libfattn_diag_nocompute.so libfattn_diag_dmaonly.so libfattn_diag_nomem.so libfattn_diag_nomem_notail.so; do
    echo "### $cfg $lib" >> gpurun_out/diag.txt
    FATTN_LIB=$lib timeout -k 10 120 $B $cfg >> gpurun_out/diag.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/diag.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
