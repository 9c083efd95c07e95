#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_split 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread  
: > gpurun_out/nt.txt
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
for c in "" "$C4" "--kv-type f16 --kv-len 2048"; do
  for spw in 0 1 2 4; do
    out=$(timeout -k 10 60 python bench.py --no-cpu-baseline --no-prefill --steps 200 --warmup 20 --spw $spw $c 2>/dev/null | grep '^{') || exit 1
    python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('%-44s spw=%s %7.2f us %.4f' % ('$c','$spw', r['kernel_ms_avg']*1e3, r['roofline']['frac']))" "$out" >> gpurun_out/nt.txt
  done
done
cat gpurun_out/nt.txt
