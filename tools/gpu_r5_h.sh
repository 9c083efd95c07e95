#!/bin/bash
# Round 5: the pipelined one-wave-per-SIMD prefill schedule (FATTN_OPT_PF_FORM
# = 4): row diagnostic, parity (bit-identical to the 8-wave body), prefill A/B.
source tools/gpu_round.sh
export TMPDIR=/tmp
run dbg_pf4p 200 python -u tools/dbg_pf4.py
run pf4p_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep"
run ab_pfp_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
run ab_pfp_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
run ab_pfp_q8r 300 python -u tools/ab_prefill.py --kv q8_0 --mask random --rounds 2 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
