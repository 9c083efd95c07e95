#!/bin/bash
# decode planner sweep (steps per wave x steps in flight) on configs 3 and 4
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 300"
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
for spw in 2 3 4 6; do for inf in 1 2 3; do
  run sw_c3_${spw}_${inf} 60 $B --spw $spw --inflight $inf
done; done
for spw in 1 2 3 4; do for inf in 1 2; do
  run sw_c4_${spw}_${inf} 60 $B $C4 --spw $spw --inflight $inf
done; done
run sw_c3_auto 60 $B
run sw_c4_auto 60 $B $C4
for f in gpurun_out/sw_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$f', j['roofline']['achieved'], j['kernel_ms_avg'])"; done
