#!/bin/bash
# Round 5, fifth GPU pass: fattn_pf4_kernel with plain row-sum adds -- its
# parity tests (bit-identical to the 8-wave form, oracle), then the prefill A/B
# of the three bodies (Q8_0 staged zero mask, f16 no mask).
source tools/gpu_round.sh
export TMPDIR=/tmp
run pf_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep or pf_staged or pf_prefill"
run ab_pf_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant pf4s1:PF_FORM=3
run ab_pf_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant pf4s1:PF_FORM=3
