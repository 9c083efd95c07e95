#!/bin/bash
# arrival stamp ahead of the publish: hand-off tests, then A/B (skip on / off / previous library)
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_ep 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -k "handoff or workspace or split_waves" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/ab.txt
for rep in 1 2 3; do
  for cfg in "" "--n-q 64 --heads 4 --kv-heads 4"; do
    echo "### $cfg NEW" >> gpurun_out/ab.txt
    timeout -k 10 120 $B $cfg >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    echo "### $cfg NOSKIP" >> gpurun_out/ab.txt
    timeout -k 10 120 $B $cfg --no-step-skip >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    echo "### $cfg PREV" >> gpurun_out/ab.txt
    FATTN_LIB=libfattn_prev.so timeout -k 10 120 $B $cfg >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/ab.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
