#!/bin/bash
# Round 4: the role-form batched decode with the raw DMA issued by all eight
# waves (product) against the build waves alone (libfattn_bissue.so), both
# without the non-temporal policy; its tests; head dim 64 role form vs the
# multi-query kernel; config 3 with / without the non-temporal policy
# (libfattn_nont.so); stamps of the product form.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4e
mkdir -p $F
run t_bdp 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bd or config5"
grep -E "passed|failed" gpurun_out/t_bdp.log | tail -2 > $F/tests_tail.txt
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10"
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
for r in 1 2; do
  run c5_all_$r 200 python bench.py $B --workload config5; line "cfg5 32h bdp all-wave issue run $r" c5_all_$r
  FATTN_LIB=libfattn_bissue.so run c5_bi_$r 200 python bench.py $B --workload config5; line "cfg5 32h bdp build-wave issue run $r" c5_bi_$r
done
run c5s2_all 200 python bench.py $B --workload config5 --heads 16 --kv-heads 16; line "cfg5 16h bdp all-wave issue" c5s2_all
FATTN_LIB=libfattn_bissue.so run c5s2_bi 200 python bench.py $B --workload config5 --heads 16 --kv-heads 16; line "cfg5 16h bdp build-wave issue" c5s2_bi
run c5q4_all 200 python bench.py $B --workload config5 --kv-type q4_0; line "cfg5-shape q4_0 all-wave issue" c5q4_all
FATTN_LIB=libfattn_bissue.so run c5q4_bi 200 python bench.py $B --workload config5 --kv-type q4_0; line "cfg5-shape q4_0 build-wave issue" c5q4_bi
run c5d64_bdp 200 python bench.py $B --workload config5 --head-dim 64 --bd 3; line "cfg5-shape D64 bdp" c5d64_bdp
run c5d64_mq 200 python bench.py $B --workload config5 --head-dim 64; line "cfg5-shape D64 planner (mq)" c5d64_mq
for r in 1 2; do
  run c3_nt_$r 200 python bench.py $B; line "cfg3 split nt run $r" c3_nt_$r
  FATTN_LIB=libfattn_nont.so run c3_nont_$r 200 python bench.py $B; line "cfg3 split no nt run $r" c3_nont_$r
done
run st_bdp 200 python tools/stamps_bd.py --form bdp --heads 32
cp gpurun_out/st_bdp.log $F/stamps_cfg5_bdp_all.txt
cat $F/tests_tail.txt $F/ab.txt $F/stamps_cfg5_bdp_all.txt
