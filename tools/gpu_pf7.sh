#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pf_ and 8waves"
: > gpurun_out/pf7.txt
for rep in 1 2; do
  for m in "" "--no-mask"; do
    out=$(timeout -k 10 60 python bench.py --n-q 4096 --steps 10 --warmup 2 --rotate 2 --no-cpu-baseline --no-prefill $m 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('%-10s %8.1f us %7.1f TF' % ('$m', r['kernel_ms_avg']*1e3, r['tflops']))" "$out" >> gpurun_out/pf7.txt
  done
done
cat gpurun_out/pf7.txt
