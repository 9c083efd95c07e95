#!/bin/bash
# merge kernel with load slots sized to the chunk count: parity + configs + kernel stats
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_m 900 python -u -m pytest tests/test_gpu_extra.py tests/test_gpu_parity.py -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/merge4.txt
for rep in 1 2; do
  for cfg in "--n-q 64" "--n-q 64 --heads 4 --kv-heads 4" "--kv-type q4_0 --kv-heads 8 --kv-len 8192"; do
    echo "### $cfg" >> gpurun_out/merge4.txt
    timeout -k 10 120 $B $cfg >> gpurun_out/merge4.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/merge4.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
run kt5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt5 -o kt -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-prefill --no-copy-peak
find gpurun_out/prof_kt5 -name "*kernel_stats.csv" -exec head -6 {} \;
