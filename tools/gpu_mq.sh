#!/bin/bash
# multi-query kernel: parity first, then the full GPU suite, then config-5 / prefill benches
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_mq 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider -k "mq or config5"
run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
run mqv 600 python tools/mq_variants.py
