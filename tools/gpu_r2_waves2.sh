#!/bin/bash
# split kernel, epilogue as a template parameter: parity, wave-count sweep, A/B against the round-start library
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_waves 600 python -u -m pytest tests/test_gpu_extra.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/ab.txt
for rep in 1 2; do
  for cfg in "" "--kv-type f16 --kv-len 2048" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "--n-q 64 --heads 4 --kv-heads 4"; do
    for w in 4 8 16; do
      echo "### $cfg --waves $w" >> gpurun_out/ab.txt
      timeout -k 10 120 $B $cfg --waves $w >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
    echo "### $cfg OLD" >> gpurun_out/ab.txt
    FATTN_LIB=libfattn_old.so timeout -k 10 120 $B $cfg >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/ab.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
