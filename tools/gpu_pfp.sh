#!/bin/bash
# pipelined prefill: timings of the schedule variants (f16 K/V prefill shape)
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill-skip --steps 20 --prefill-kv f16"
B="python bench.py --no-cpu-baseline --steps 20 --prefill-kv f16"
run pf_base 120 $B --pf-pipe 1
run pf_pipe 120 $B --pf-pipe 2
run pf_pipe_s0 120 $B --pf-pipe 2 --pf-stagger 0
run pf_pipe_s1 120 $B --pf-pipe 2 --pf-stagger 3
FATTN_LIB=libfattn_pfp_r4r8.so run pf_pipe_r4r8 120 $B --pf-pipe 2
FATTN_LIB=libfattn_pfp_r8r16.so run pf_pipe_r8r16 120 $B --pf-pipe 2
FATTN_LIB=libfattn_pfp_r8r16.so run pf_pipe_r8r16_s0 120 $B --pf-pipe 2 --pf-stagger 0
run pf_base_s0 120 $B --pf-pipe 1 --pf-stagger 0
for f in gpurun_out/pf_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)['prefill']; print('$f', j['kernel'], j['kernel_ms_avg'], j['roofline']['achieved'], j['roofline']['frac'])"; done
