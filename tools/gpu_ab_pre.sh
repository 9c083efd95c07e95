#!/bin/bash
# A/B on one box: in-kernel dequant vs f16 pre-pass, random and causal masks, alternating
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --steps 20"
for r in 1 2 3; do
  run ab_ink_r$r 120 $B --pf-dequant 1
  run ab_pre_r$r 120 $B --pf-dequant 2
  run ab_ink_c$r 120 $B --pf-dequant 1 --prefill-causal
  run ab_pre_c$r 120 $B --pf-dequant 2 --prefill-causal
done
for f in gpurun_out/ab_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l)['prefill']; print('$(basename $f .log)', j['workload'], j['kernel_ms_avg'], j['roofline']['frac'])"; done
