#!/bin/bash
# rocprofv3 kernel-trace summary + PMC (FETCH_SIZE, WRITE_SIZE in separate passes) of the default bench
source tools/gpu_round.sh
export TMPDIR=/tmp
run prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
run prof_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline
run prof_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline
