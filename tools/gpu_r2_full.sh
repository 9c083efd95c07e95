#!/bin/bash
# whole GPU suite, then the bench line on the default plan
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | head -30
run bench1 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 4
grep '^{' gpurun_out/bench1.log > gpurun_out/bench1.json || true
