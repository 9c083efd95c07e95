#!/bin/bash
# decode geometry sweep + stamp timelines (config 3 and 4)
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --steps 100 --warmup 10"
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
run st_c3 120 python tools/stamps.py
run st_c3_nc 120 python tools/stamps.py --nocompute
run st_c4 120 python tools/stamps.py $C4
run st_c3_s4i4 120 python tools/stamps.py --spw 4 --inflight 4
for cfg in "1 1" "2 2" "4 2" "4 3" "4 4" "8 2" "8 4"; do set -- $cfg
  run sw_c3_s$1_i$2 120 $B --spw $1 --inflight $2
done
for cfg in "1 1" "2 2" "4 2" "4 4" "8 2"; do set -- $cfg
  run sw_c4_s$1_i$2 120 $B $C4 --spw $1 --inflight $2
done
FATTN_LIB=libfattn_nt.so run nt_c3 120 $B
FATTN_LIB=libfattn_nt.so run nt_c3_s4i4 120 $B --spw 4 --inflight 4
for f in gpurun_out/sw_*.log gpurun_out/nt_*.log; do
  python3 -c "
import sys,json
for l in open('$f'):
    if l.startswith('{'):
        r=json.loads(l); print('$f', r['kernel_ms_avg']*1e3, r['roofline']['frac'])"
done > gpurun_out/sweep_summary.txt
