#!/bin/bash
# config 3 planner sweep with the wave-level merge, then the round-end set
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 300"
for spw in 4 5 8; do for inf in 1 2 3; do
  run sw3_c3_${spw}_${inf} 60 $B --spw $spw --inflight $inf
done; done
for f in gpurun_out/sw3_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$f', j['roofline']['achieved'], j['kernel_ms_avg'])"; done
