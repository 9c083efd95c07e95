#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
run st_c3_s1_tag 120 python tools/stamps.py --spw 1 --inflight 1
run st_c3_s1_untag 120 python tools/stamps.py --spw 1 --inflight 1 --untagged
run st_c4_s1_tag 120 python tools/stamps.py --spw 1 --inflight 1 $C4
run st_c4_s1_untag 120 python tools/stamps.py --spw 1 --inflight 1 --untagged $C4
