#!/bin/bash
# pipelined prefill: parity, then timings pipe on/off (f16 K/V and q8_0 pre-pass)
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pf"
B="python bench.py --no-cpu-baseline --steps 20"
run pf_f16_pipe 120 $B --prefill-kv f16
run pf_pre_pipe 120 $B --pf-dequant 2
run pf_ink 120 $B --pf-dequant 1
run pf_f16_pipe2 120 $B --prefill-kv f16
for f in gpurun_out/pf_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)['prefill']; print('$f', j['kernel'], j['kernel_ms_avg'], j['roofline']['achieved'], j['roofline']['frac'])"; done
