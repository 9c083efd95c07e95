#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 300"
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
C2="--kv-type f16 --kv-len 2048"
for r in 1 2 3; do
  run ek_c3_new_$r 60 $B
  FATTN_LIB=libfattn_noearlyk.so run ek_c3_old_$r 60 $B
  run ek_c4_new_$r 60 $B $C4
  FATTN_LIB=libfattn_noearlyk.so run ek_c4_old_$r 60 $B $C4
  run ek_c2_new_$r 60 $B $C2
  FATTN_LIB=libfattn_noearlyk.so run ek_c2_old_$r 60 $B $C2
done
for f in gpurun_out/ek_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$(basename $f .log)', j['kernel_ms_avg'])"; done
