#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pf or wave_merge"
B="python bench.py --no-cpu-baseline --steps 20"
run pfc_q8 120 $B --prefill-causal
run pfc_f16 120 $B --prefill-causal --prefill-kv f16
run pfc_q8_rand 120 $B
for f in gpurun_out/pfc_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)['prefill']; print('$f', j['workload'], j['kernel_ms_avg'], j['roofline']['achieved'], j['roofline']['frac'])"; done
