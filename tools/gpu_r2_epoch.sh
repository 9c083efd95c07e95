#!/bin/bash
# epoch-stamped arrival words: whole GPU suite, then A/B of the decode configs against libfattn_prev.so
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | head -30
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/ab.txt
for rep in 1 2 3; do
  for cfg in "" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "--n-q 64 --heads 4 --kv-heads 4"; do
    echo "### $cfg NEW" >> gpurun_out/ab.txt
    timeout -k 10 120 $B $cfg >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    echo "### $cfg PREV" >> gpurun_out/ab.txt
    FATTN_LIB=libfattn_prev.so timeout -k 10 120 $B $cfg >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/ab.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
