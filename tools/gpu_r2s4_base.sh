#!/bin/bash
# round-2 re-entry baseline: GPU suite, bench line, HBM probe
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread
run bench1 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 4
grep '^{' gpurun_out/bench1.log > gpurun_out/bench1.json || true
run hbm_probe 120 tools/_build/hbm_probe
cat gpurun_out/hbm_probe.log
