#!/bin/bash
# parity suite + decode bench lines for configs 3, 4, 2 (no CPU baseline, no prefill)
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python bench.py --no-cpu-baseline --no-prefill --steps 500"
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run bench_c3 120 $B
run bench_c3b 120 $B
run bench_c4 120 $B --kv-type q4_0 --kv-heads 8 --kv-len 8192
run bench_c2 120 $B --kv-type f16 --kv-len 2048
for f in gpurun_out/bench_c*.log; do grep -h '^{' $f | python3 -c "
import sys, json
for l in sys.stdin:
    j = json.loads(l); print('$f', j['roofline']['achieved'], j['roofline']['frac'], j['kernel_ms_avg'])"; done
