#!/bin/bash
# Round 5: per-phase cycle stamps of the pipelined prefill body (stamps build),
# f16 no mask and Q8_0 staged random mask, and of the 8-wave body beside it.
source tools/gpu_round.sh
export TMPDIR=/tmp
run st_pf4p_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16
run st_pf4p_q8 200 python -u tools/pf_stamps.py --kv-type q8_0
run st_pf8_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16 --form 1
