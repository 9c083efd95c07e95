#!/bin/bash
# end-of-round: GPU parity suite, default bench, rocprof kernel trace, FETCH/WRITE PMC passes
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run bench 300 python bench.py
source tools/gpu_prof.sh
