#!/bin/bash
# A/B/C on config 3 and config 5 shard: previous commit, step-skip commit, working tree
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_ep 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/abc.txt
for rep in 1 2 3; do
  for cfg in "" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "--n-q 64 --heads 4 --kv-heads 4" "--mask-live 0.3" "--kv-len 32768 --heads 8 --kv-heads 8 --mask-live 0.3"; do
    for lib in libfattn_prev.so libfattn.so; do
      echo "### $cfg $lib" >> gpurun_out/abc.txt
      FATTN_LIB=$lib timeout -k 10 120 $B $cfg >> gpurun_out/abc.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/abc.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
