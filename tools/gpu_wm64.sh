#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-prefill --steps 300"
for spw in 2 3 4; do for inf in 1 2; do
  run sw4_c3_${spw}_${inf} 60 $B --spw $spw --inflight $inf
done; done
run sw4_c3_auto 60 $B
for f in gpurun_out/sw4_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$f', j['roofline']['achieved'], j['kernel_ms_avg'])"; done
