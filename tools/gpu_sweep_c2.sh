#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 300 --kv-type f16 --kv-len 2048"
run c2_auto 60 $B
for spw in 1 2 3 4; do for inf in 1 2; do run c2_${spw}_${inf} 60 $B --spw $spw --inflight $inf; done; done
run c2_auto2 60 $B
for f in gpurun_out/c2_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$(basename $f .log)', j['roofline']['achieved'], j['kernel_ms_avg'])"; done
