#!/bin/bash
export TMPDIR=/tmp
: > gpurun_out/pf6.txt
for lib in libfattn.so libfattn_pf4nosgb.so; do
  for w in 4; do
    out=$(FATTN_LIB=$lib timeout -k 10 60 python bench.py --n-q 4096 --steps 10 --warmup 2 --rotate 2 --no-cpu-baseline --no-prefill --pf-waves $w 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('%s waves=%s %8.1f us %7.1f TF' % ('$lib','$w', r['kernel_ms_avg']*1e3, r['tflops']))" "$out" >> gpurun_out/pf6.txt
  done
done
cat gpurun_out/pf6.txt
