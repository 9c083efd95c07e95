#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 300"
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
for r in a b; do for pr in 0 1 2; do
  run pr_c3_${pr}_$r 60 $B --split-prio $pr
  run pr_c4_${pr}_$r 60 $B $C4 --split-prio $pr
  run pr_c2_${pr}_$r 60 $B --kv-type f16 --kv-len 2048 --split-prio $pr
done; done
for f in gpurun_out/pr_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$f', j['roofline']['achieved'], j['kernel_ms_avg'])"; done
