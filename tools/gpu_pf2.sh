#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_pf 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "pf_"
bash tools/gpu_pfm.sh
