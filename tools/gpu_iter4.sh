#!/bin/bash
# decode: fixed overhead (dec diag 3), memory-only, compute-only, split
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_dec 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -x -q -p no:cacheprovider --timeout 180 --timeout-method thread -k "config or sweep or wave_merge or rescale or masked or chunking or determin or dec_kernel"
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/ab.txt
for rep in 1 2; do
  for v in "--dec 1" "--dec 2 --dec-compute 8" "--dec 2 --dec-diag 3" "--dec 2 --dec-diag 3 --dec-compute 8" "--dec 2 --dec-diag 1" "--dec 2 --dec-diag 2" "--dec 2 --dec-diag 2 --dec-compute 8"; do
    echo "### $v" >> gpurun_out/ab.txt
    timeout -k 10 120 $B $v >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/ab.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*/  kernel_ms \1 median \2 frac \3/'
