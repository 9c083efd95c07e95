#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
: > gpurun_out/pf3.txt
for rep in 1 2 3; do
for st in 1 0; do
  for m in "" "--no-mask"; do
    out=$(timeout -k 10 60 python bench.py --n-q 4096 --steps 10 --warmup 2 --rotate 2 --no-cpu-baseline --pf-stagger $st $m 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('stagger=%s %-10s %8.1f us %7.1f TF' % ('$st','$m', r['kernel_ms_avg']*1e3, r['tflops']))" "$out" >> gpurun_out/pf3.txt
  done
done
done
cat gpurun_out/pf3.txt
