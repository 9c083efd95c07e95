#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
: > gpurun_out/pfm.txt
for lib in libfattn.so libfattn_mq_nocomp.so libfattn_pf_nosm.so libfattn_mq_nodeq.so; do
  for m in "" "--no-mask"; do
    out=$(FATTN_LIB=$lib timeout -k 10 60 python bench.py --n-q 4096 --steps 5 --warmup 1 --rotate 2 --no-cpu-baseline $m 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('%-24s %-10s %8.1f us %7.1f TF' % ('$lib','$m', r['kernel_ms_avg']*1e3, r['tflops']))" "$out" >> gpurun_out/pfm.txt
  done
done
cat gpurun_out/pfm.txt
