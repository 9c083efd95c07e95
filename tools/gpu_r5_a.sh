#!/bin/bash
# Round 5, first GPU pass: the GPU suite (KAT through the kernels, the world-1
# RCCL bench path, speculative merge / XCD order, prefill staging and the
# one-wave-per-SIMD body), then same-box A/Bs (config 3 options; prefill forms).
source tools/gpu_round.sh
export TMPDIR=/tmp
run tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread
run ab_cfg3 300 python -u tools/ab_decode.py --workload config3 --rounds 6 \
    --variant base: --variant spec:SPLIT_SPEC=2 --variant xcd:SPLIT_XCD=2 --variant spec_xcd:SPLIT_SPEC=2,SPLIT_XCD=2
run ab_pf_zero 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 2 \
    --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant inkernel:PF_STAGE=1,PF_FORM=1
