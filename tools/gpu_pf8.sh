#!/bin/bash
# prefill: phase stamps (f16, q8_0 in-kernel) and the XCD-grouped order
source tools/gpu_round.sh
export TMPDIR=/tmp
run st_f16 120 python tools/pf_stamps.py --kv-type f16
run st_q8 120 python tools/pf_stamps.py --kv-type q8_0
B="python bench.py --no-cpu-baseline --steps 20"
run pf_f16_s2 120 $B --prefill-kv f16 --pf-stagger 2
run pf_f16_s6 120 $B --prefill-kv f16 --pf-stagger 6
run pf_pre_s2 120 $B --pf-dequant 2 --pf-stagger 2
run pf_pre_s6 120 $B --pf-dequant 2 --pf-stagger 6
run pf_ink_s6 120 $B --pf-dequant 1 --pf-stagger 6
run pf_f16_s2b 120 $B --prefill-kv f16 --pf-stagger 2
run pf_f16_s6b 120 $B --prefill-kv f16 --pf-stagger 6
cat gpurun_out/st_f16.log gpurun_out/st_q8.log | grep -v amdgpu.ids
for f in gpurun_out/pf_*_s*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)['prefill']; print('$f', j['kernel'], j['kernel_ms_avg'], j['roofline']['achieved'], j['roofline']['frac'])"; done
