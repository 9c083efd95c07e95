#!/bin/bash
# decode grid shapes: many small workgroups vs one 16-wave workgroup per CU
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/grid.txt
for rep in 1 2; do
  for v in "--waves 16" "--waves 4 --spw 1" "--waves 8 --spw 1" "--waves 4 --spw 2" "--waves 8 --spw 2 --inflight 1" \
           "--kv-type q4_0 --kv-heads 8 --kv-len 8192 --waves 4 --spw 1" "--kv-type q4_0 --kv-heads 8 --kv-len 8192 --waves 4" \
           "--n-q 64 --heads 4 --kv-heads 4 --waves 4 --spw 1" "--n-q 64 --heads 4 --kv-heads 4 --waves 4"; do
    echo "### $v" >> gpurun_out/grid.txt
    timeout -k 10 120 $B $v >> gpurun_out/grid.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/grid.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
