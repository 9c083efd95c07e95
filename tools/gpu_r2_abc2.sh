#!/bin/bash
# config 3: previous commit vs working tree, step skip on / off
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
rm -f gpurun_out/abc.txt
for rep in 1 2 3 4; do
  for v in "prev" "new" "noskip"; do
    echo "### $v" >> gpurun_out/abc.txt
    case $v in
      prev) FATTN_LIB=libfattn_prev.so timeout -k 10 120 $B >> gpurun_out/abc.txt 2>&1 ;;
      new) timeout -k 10 120 $B >> gpurun_out/abc.txt 2>&1 ;;
      noskip) timeout -k 10 120 $B --no-step-skip >> gpurun_out/abc.txt 2>&1 ;;
    esac || { echo "STOP rc=$?"; exit 1; }
  done
done
grep -E "###|kernel_ms_avg" gpurun_out/abc.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3/'
