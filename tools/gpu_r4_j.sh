#!/bin/bash
# Round 4: role-form batched decode -- each compute wave's mask DMA for tile
# s + 2 issued before tile s's compute (product) against after it
# (libfattn_mlate.so, FATTN_BDP_MASK_LATE); its tests; the product's stamps;
# prefill zero-mask tiles without mask DMA (libfattn_zdma.so: with it).
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
# prefill, quantised K/V: zero-mask tiles' mask DMA not issued (product) against
# issued through an offset past the descriptor (libfattn_zdma.so, FATTN_PF_ZERO_DMA)
run t_pf 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "pf or prefill"
grep -E "passed|failed" gpurun_out/t_pf.log | tail -2 >> $F/tests_tail.txt
for r in 1 2 3; do
  run pfz_skip_$r 150 python bench.py --prefill-only; line "prefill q8_0 zero mask, zero tiles' mask DMA skipped run $r" pfz_skip_$r
  FATTN_LIB=libfattn_zdma.so run pfz_oob_$r 150 python bench.py --prefill-only; line "prefill q8_0 zero mask, zero tiles' mask DMA out of bounds run $r" pfz_oob_$r
done
run pfc_skip 150 python bench.py --prefill-only --prefill-mask causal; line "prefill q8_0 causal, skipped" pfc_skip
FATTN_LIB=libfattn_zdma.so run pfc_oob 150 python bench.py --prefill-only --prefill-mask causal; line "prefill q8_0 causal, out of bounds" pfc_oob
run st_bdp 200 python tools/stamps_bd.py --form bdp --heads 32
cp gpurun_out/st_bdp.log $F/stamps_cfg5_bdp.txt
cat $F/tests_tail.txt $F/ab.txt $F/stamps_cfg5_bdp.txt
