#!/bin/bash
# head dims 80 / 96 parity, then the lagged-issue sweep
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_d96 600 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --maxfail 20 --timeout 120 --timeout-method thread -k "D80 or D96"
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_d96.log | head -30
bash tools/gpu_r2_lag.sh
