#!/bin/bash
# Round 4: role-form batched decode -- each compute wave's mask DMA for tile
# s + 2 issued before tile s's compute (product) against after it
# (libfattn_mlate.so, FATTN_BDP_MASK_LATE); its tests; the product's stamps.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4j
mkdir -p $F
run t_bdp 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bdp or bd_ or xcd"
grep -E "passed|failed" gpurun_out/t_bdp.log | tail -2 > $F/tests_tail.txt
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
for r in 1 2 3; do
  run c5_me_$r 150 python bench.py $B; line "cfg5 bdp mask issued before the compute run $r" c5_me_$r
  FATTN_LIB=libfattn_mlate.so run c5_ml_$r 150 python bench.py $B; line "cfg5 bdp mask issued after the compute run $r" c5_ml_$r
done
run c5s2_me 150 python bench.py $B --heads 16 --kv-heads 16; line "cfg5 16h bdp mask before" c5s2_me
FATTN_LIB=libfattn_mlate.so run c5s2_ml 150 python bench.py $B --heads 16 --kv-heads 16; line "cfg5 16h bdp mask after" c5s2_ml
run st_bdp 200 python tools/stamps_bd.py --form bdp --heads 32
cp gpurun_out/st_bdp.log $F/stamps_cfg5_bdp.txt
cat $F/tests_tail.txt $F/ab.txt $F/stamps_cfg5_bdp.txt
