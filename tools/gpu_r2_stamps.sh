#!/bin/bash
# phase stamps of the split kernel at 16 / 8 / 4 waves; same-box A/B against the previous library
source tools/gpu_round.sh
export TMPDIR=/tmp
run st16 60 python tools/stamps.py --waves 16
run st8 60 python tools/stamps.py --waves 8
run st4 60 python tools/stamps.py --waves 4
run st2f16 60 python tools/stamps.py --kv-type f16 --kv-len 2048
run st4q4 60 python tools/stamps.py --kv-type q4_0 --kv-heads 8 --kv-len 8192
cat gpurun_out/st16.log gpurun_out/st8.log gpurun_out/st4.log gpurun_out/st2f16.log gpurun_out/st4q4.log
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200"
rm -f gpurun_out/ab.txt
for rep in 1 2 3; do
  for lib in libfattn_old.so libfattn.so; do
    echo "### $lib" >> gpurun_out/ab.txt
    FATTN_LIB=$lib timeout -k 10 120 $B >> gpurun_out/ab.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/ab.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
