#!/bin/bash
# lagged issue: parity, then decode configs
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_waves 600 python -u -m pytest tests/test_gpu_extra.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k split_waves
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/lag.txt
for rep in 1 2; do
  for v in "--waves 8 --spw 2 --inflight 1" "--waves 8 --spw 2 --lag 1" "--waves 4 --lag 1" "--waves 4 --spw 4 --inflight 3 --lag 1" "--waves 16" \
           "--waves 8 --spw 4 --inflight 1" "--waves 4 --spw 8 --inflight 1" \
           "--kv-type f16 --kv-len 2048 --waves 4 --spw 2 --lag 1" "--kv-type f16 --kv-len 2048 --waves 8" \
           "--kv-type q4_0 --kv-heads 8 --kv-len 8192 --waves 4 --lag 1" "--kv-type q4_0 --kv-heads 8 --kv-len 8192 --waves 4 --spw 4 --inflight 1" \
           "--n-q 64 --heads 4 --kv-heads 4 --waves 4 --lag 1" "--n-q 64 --heads 4 --kv-heads 4 --waves 4 --spw 4 --inflight 1"; do
    echo "### $v" >> gpurun_out/lag.txt
    timeout -k 10 120 $B $v >> gpurun_out/lag.txt 2>&1 || echo "rc=$? for $v" >> gpurun_out/lag.txt
  done
done
grep -E "###|kernel_ms_avg|rc=" gpurun_out/lag.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
