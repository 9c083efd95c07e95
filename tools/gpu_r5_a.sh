#!/bin/bash
# Round 5, first GPU pass: the GPU suite (KAT through the kernels, the world-1
# RCCL bench path, the speculative merge / XCD order parity), a config-3 A/B of
# the two new split-kernel options, and the default bench line.
source tools/gpu_round.sh
export TMPDIR=/tmp
run tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
run ab_cfg3 300 python -u tools/ab_decode.py --workload config3 --rounds 6 \
    --variant base: --variant spec:SPLIT_SPEC=2 --variant xcd:SPLIT_XCD=2 --variant spec_xcd:SPLIT_SPEC=2,SPLIT_XCD=2
run bench 400 python -u bench.py
