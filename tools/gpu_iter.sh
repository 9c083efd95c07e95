#!/bin/bash
# One measure pass: parity, chunk sweep, stamp timelines, kernel-trace profile, default bench line.
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
run sweep 600 python tools/sweep_chunk.py
run stamps_auto 200 python tools/stamps.py
run nocomp_auto 200 python tools/stamps.py --nocompute
run prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline
run bench 600 python bench.py --cpu-seconds 3
