#!/bin/bash
# full round: GPU parity suite, default bench (decode + prefill + cpu baseline), rocprof kernel trace
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run bench 300 python bench.py
run prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
