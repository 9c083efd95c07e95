#!/bin/bash
# ping-pong prefill: parity (both schedules), then the prefill shape in both
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 600 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --maxfail 10 --timeout 120 --timeout-method thread -k "pf_"
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_pf.log | head -30
B="python bench.py --no-cpu-baseline --no-scale-ref --no-copy-peak --steps 20"
rm -f gpurun_out/pf2.txt
for rep in 1 2; do
  for v in "--pf-pipe 1" "--pf-pipe 2" "--pf-pipe 2 --prefill-causal" "--pf-pipe 1 --prefill-causal" "--pf-pipe 2 --prefill-kv q4_0"; do
    echo "### $v" >> gpurun_out/pf2.txt
    timeout -k 10 120 $B $v >> gpurun_out/pf2.txt 2>&1 || echo "rc=$? $v" >> gpurun_out/pf2.txt
  done
done
python3 - <<'PY'
import json
for l in open('gpurun_out/pf2.txt'):
    if l.startswith('###') or l.startswith('rc='): print(l.strip())
    elif l.startswith('{'):
        d=json.loads(l); p=d['prefill']; print('  prefill', p['kernel_ms_avg'], p['roofline']['frac'], p['kernel'][:60])
PY
