#!/bin/bash
# Round 5, sixth GPU pass: pf4 parity after the contraction fix; same-box A/B of
# the multi-row split merges (second launch vs last-arriving workgroup, XCD
# order, chunk size) on config 4 and the config-5 4- and 8-rank shards.
source tools/gpu_round.sh
export TMPDIR=/tmp
run pf4_tests 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "pf4"
V="--variant base: --variant fused:SPLIT_MERGE=1 --variant xcd:SPLIT_XCD=2 --variant fx:SPLIT_MERGE=1,SPLIT_XCD=2"
run ab_cfg4 300 python -u tools/ab_decode.py --workload config4 --rounds 5 $V \
    --variant fx512:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=512 --variant fx1024:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=1024
run ab_s8 300 python -u tools/ab_decode.py --workload config5_s8 --rounds 5 $V \
    --variant fx512:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=512
run ab_s4 300 python -u tools/ab_decode.py --workload config5_s4 --rounds 5 $V \
    --variant fx512:SPLIT_MERGE=1,SPLIT_XCD=2,kv_chunk=512
# bdp image swizzles (round 5): parity, then config 5 new vs old swizzles (two libraries, alternating processes)
run bdp_tests 300 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu -k "bdp"
FATTN_LIB=libfattn_raw64.so run bdp_tests_raw64 300 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu -k "bdp"
for i in 1 2; do
  run ab_c5_new_$i 200 python -u tools/ab_decode.py --workload config5 --rounds 3 --variant new:
  run ab_c5_old_$i 200 python -u tools/ab_decode.py --workload config5 --rounds 3 --variant old: --lib libfattn_oldswz.so
  run ab_c5_raw64_$i 200 python -u tools/ab_decode.py --workload config5 --rounds 3 --variant raw64: --lib libfattn_raw64.so
done
run nccl_world1 400 python -u -m pytest tests/test_rehearsal.py -x -q --timeout 300 --timeout-method thread -m gpu -k "nccl"
# D = 256 (verdict r04 missing 2): batched decode (config-5 shape) multi-query vs split kernel; prefill
run ab_d256_dec 300 python -u tools/ab_decode.py --workload config5 --D 256 --rounds 3 --variant mq: --variant split:MQ_DISABLE=1
run ab_d256_pf 300 python -u tools/ab_prefill.py --kv q8_0 --mask zero --D 256 --H 16 --rounds 2 --variant auto:
run ab_d256_pf16 300 python -u tools/ab_prefill.py --kv f16 --mask none --D 256 --H 16 --rounds 2 --variant auto:
