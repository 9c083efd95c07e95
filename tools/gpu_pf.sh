#!/bin/bash
# prefill kernel: parity first, then prefill / config-5 timings vs the multi-query kernel
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "pf_"
run pf_bench 120 python bench.py --n-q 4096 --steps 5 --warmup 1 --rotate 2 --no-cpu-baseline
run pf_bench_mq 120 python bench.py --n-q 4096 --steps 5 --warmup 1 --rotate 2 --no-cpu-baseline --pf 1
run pf_bench_q4 120 python bench.py --n-q 4096 --steps 5 --warmup 1 --rotate 2 --no-cpu-baseline --kv-type q4_0
for f in pf_bench pf_bench_mq pf_bench_q4; do grep -h '^{' gpurun_out/$f.log | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print('$f', r['kernel_ms_avg']*1e3, 'us', r['tflops'], 'TF', r['roofline'])"; done
