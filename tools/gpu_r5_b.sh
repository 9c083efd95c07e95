#!/bin/bash
# Round 5, second GPU pass: the one-wave-per-SIMD prefill body after the
# branch-free / immediate-offset rework, the XCD-order default, then a
# same-box prefill A/B.
source tools/gpu_round.sh
export TMPDIR=/tmp
run tests_sel 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "pf or xcd or row_merge or workspace_not_zeroed or kat or nccl"
run ab_pf_zero 400 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 \
    --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant inkernel:PF_STAGE=1,PF_FORM=1
run ab_pf_random 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 \
    --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2
