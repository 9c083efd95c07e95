#!/bin/bash
# step skip from 4 steps per wave: parity, then config 3 and long-KV masked A/B
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_ep 600 python -u -m pytest tests/test_gpu_extra.py -k "split_waves or step_skip or workspace" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/abc.txt
for rep in 1 2 3; do
  for cfg in "" "--kv-len 32768 --heads 8 --kv-heads 8 --mask-live 0.3" "--kv-len 32768 --heads 8 --kv-heads 8"; do
    for v in prev new; do
      echo "### $cfg $v" >> gpurun_out/abc.txt
      if [ $v = prev ]; then FATTN_LIB=libfattn_prev.so timeout -k 10 120 $B $cfg >> gpurun_out/abc.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
      else timeout -k 10 120 $B $cfg >> gpurun_out/abc.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }; fi
    done
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/abc.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
