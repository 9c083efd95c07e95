#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 100 --n-q 64"
run c5_h4 60 $B --heads 4
run c5_h4_split 60 $B --heads 4 --no-mq
run c5_h4_split_spw2 60 $B --heads 4 --no-mq --spw 2
run c5_h4_split_spw1 60 $B --heads 4 --no-mq --spw 1
run c5_h32 60 $B
run c5_h32_split 60 $B --no-mq
for f in gpurun_out/c5_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$f', j['config']['workload'], j['roofline']['achieved'], j['roofline']['frac'], j['kernel_ms_avg'], j['roofline']['kernel'])"; done
