#!/bin/bash
# session-2 state check: full GPU parity suite, default bench, config-5 / prefill benches, rocprof trace
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run bench 300 python bench.py
run bench_c4 200 python bench.py --kv-type q4_0 --heads 32 --kv-heads 8 --kv-len 8192 --no-cpu-baseline
run bench_c2 200 python bench.py --kv-type f16 --kv-len 2048 --no-cpu-baseline
run mqv 600 python tools/mq_variants.py
run prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
