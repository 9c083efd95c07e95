#!/bin/bash
# Round 4: the role-form batched-decode kernel with its raw ring sized by the
# LDS (Q8_0 4 tiles, Q4_0 5) -- its tests, then config 5 alternating the
# product library, the 3-tile ring (libfattn_nr3.so) and a no-dequantisation
# diagnostic build (libfattn_nodeq.so: build waves only move bytes), and the
# phase stamps of the product form; libfattn_nont.so: K/V DMA without the
# non-temporal policy.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4d
mkdir -p $F
run t_bdp 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bd or config5"
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
for r in 1 2; do
  run c5_nr4_$r 200 python bench.py $B; line "cfg5 32h bdp nRaw 4 run $r" c5_nr4_$r
  FATTN_LIB=libfattn_nr3.so run c5_nr3_$r 200 python bench.py $B; line "cfg5 32h bdp nRaw 3 run $r" c5_nr3_$r
  FATTN_LIB=libfattn_nodeq.so run c5_nodeq_$r 200 python bench.py $B; line "cfg5 32h bdp no dequant (diag) run $r" c5_nodeq_$r
  run c5_bd_$r 200 python bench.py $B --bd 2; line "cfg5 32h bd (all waves) run $r" c5_bd_$r
  FATTN_LIB=libfattn_nont.so run c5_nont_$r 200 python bench.py $B; line "cfg5 32h bdp nRaw 4, K/V DMA without nt run $r" c5_nont_$r
done
run c5s2_nr4 200 python bench.py $B --heads 16 --kv-heads 16; line "cfg5 16h bdp nRaw 4" c5s2_nr4
FATTN_LIB=libfattn_nr3.so run c5s2_nr3 200 python bench.py $B --heads 16 --kv-heads 16; line "cfg5 16h bdp nRaw 3" c5s2_nr3
run c5q4_nr5 200 python bench.py $B --kv-type q4_0; line "cfg5-shape q4_0 bdp nRaw 5" c5q4_nr5
FATTN_LIB=libfattn_nr3.so run c5q4_nr3 200 python bench.py $B --kv-type q4_0; line "cfg5-shape q4_0 bdp nRaw 3" c5q4_nr3
run st_bdp 200 python tools/stamps_bd.py --form bdp --heads 32
cp gpurun_out/st_bdp.log $F/stamps_cfg5_bdp_nr4.txt
grep -E "passed|failed" gpurun_out/t_bdp.log | tail -2 > $F/tests_tail.txt
cat $F/tests_tail.txt $F/ab.txt $F/stamps_cfg5_bdp_nr4.txt
