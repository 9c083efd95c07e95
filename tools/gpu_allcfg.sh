#!/bin/bash
# every BASELINE config's bench line plus the prefill variants, final tree
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --steps 200"
run all_c2 120 $B --no-prefill --kv-type f16 --kv-len 2048
run all_c3 120 $B
run all_c4 120 $B --no-prefill --kv-type q4_0 --kv-heads 8 --kv-len 8192
run all_c5_h4 120 $B --no-prefill --n-q 64 --heads 4
run all_c5_h32 120 $B --no-prefill --n-q 64
run all_pf_q8_causal 120 $B --prefill-causal
run all_pf_f16 120 $B --prefill-kv f16
run all_pf_f16_causal 120 $B --prefill-kv f16 --prefill-causal
run all_pf_q4 120 $B --prefill-kv q4_0
for f in gpurun_out/all_*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); r = j['roofline']; pf = j.get('prefill')
    print('$(basename $f .log)', j['config']['workload'], r['kernel'], j['kernel_ms_avg'], r['achieved'], r['frac'],
          '| prefill', (pf['workload'], pf['kernel_ms_avg'], pf['roofline']['achieved'], pf['roofline']['frac']) if pf else '-')"; done
