#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
: > gpurun_out/pf4.txt
for rep in 1 2; do
for st in 0 1 2 3; do
    out=$(timeout -k 10 60 python bench.py --n-q 4096 --steps 10 --warmup 2 --rotate 2 --no-cpu-baseline --no-prefill --pf-stagger $st 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('stagger=%s %8.1f us %7.1f TF' % ('$st', r['kernel_ms_avg']*1e3, r['tflops']))" "$out" >> gpurun_out/pf4.txt
done
done
cat gpurun_out/pf4.txt
