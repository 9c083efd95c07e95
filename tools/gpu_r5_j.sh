#!/bin/bash
# Round 5: pipelined prefill with its operand reads streamed inside the steps:
# parity, stamps, same-box A/B against the 8-wave body.
source tools/gpu_round.sh
export TMPDIR=/tmp
run pf4p_tests 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4 or pf_sweep or pf_prefill or pf_staged"
run st_pf4p_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16
run st_pf4p_q8 200 python -u tools/pf_stamps.py --kv-type q8_0
run ab_pfp_f16 300 python -u tools/ab_prefill.py --kv f16 --mask none --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
run ab_pfp_q8 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --rounds 3 --variant pf8:PF_FORM=1 --variant pf4p:PF_FORM=4
