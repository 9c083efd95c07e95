#!/bin/bash
# multi-query kernel vs split kernel (+ second-launch merge) on batched-decode shapes
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_g 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --rotate 4"
rm -f gpurun_out/mq.txt
for cfg in "--n-q 64 --heads 32 --kv-heads 8" "--n-q 128 --heads 32 --kv-heads 8" "--n-q 256" "--n-q 64 --heads 32 --kv-heads 8 --kv-type q4_0" "--n-q 256 --heads 8 --kv-heads 8 --kv-len 8192"; do
  for v in "" "--no-mq"; do
    echo "### $cfg $v" >> gpurun_out/mq.txt
    timeout -k 10 120 $B $cfg $v >> gpurun_out/mq.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/mq.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
