#!/bin/bash
# Round 5, second GPU pass: the one-wave-per-SIMD prefill body (fattn_pf4.h)
# -- parity first (bit-identical to the 8-wave body, the prefill sweeps over
# all three forms), then a same-box prefill A/B.
source tools/gpu_round.sh
export TMPDIR=/tmp
run tests_pf 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "pf"
run ab_pf_zero 400 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 \
    --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant inkernel:PF_STAGE=1,PF_FORM=1
run ab_pf_random 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 \
    --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2
run ab_pf_f16 300 python -u tools/ab_prefill.py --kv f16 --mask zero --rounds 2 \
    --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2
