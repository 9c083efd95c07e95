#!/bin/bash
# prefill: parity (pf tests), then the prefill shape in-kernel dequant vs f16 pre-pass vs f16 K/V
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pf"
B="python bench.py --no-cpu-baseline --steps 50"
run pf_inkernel 120 $B --pf-dequant 1
run pf_pre 120 $B --pf-dequant 2
run pf_f16 120 $B --prefill-kv f16
run pf_inkernel2 120 $B --pf-dequant 1
run pf_pre2 120 $B --pf-dequant 2
for f in gpurun_out/pf_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)['prefill']; print('$f', j['kernel'], j['kernel_ms_avg'], j['roofline']['achieved'], j['roofline']['frac'])"; done
