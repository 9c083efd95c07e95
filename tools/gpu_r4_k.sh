#!/bin/bash
# Round 4: role-form build waves -- raw reads, DMA issue, conversion + image
# writes (product) against raw reads, conversion + image writes, then the DMA
# issue (libfattn_deqfirst.so, built from a patched copy of the sources).
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4k
mkdir -p $F
FATTN_LIB=libfattn_deqfirst.so run t_bdp 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bdp"
grep -E "passed|failed" gpurun_out/t_bdp.log | tail -2 > $F/tests_tail.txt
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
for r in 1 2 3; do
  run c5_p_$r 150 python bench.py $B; line "cfg5 bdp reads, issue, convert+write run $r" c5_p_$r
  FATTN_LIB=libfattn_deqfirst.so run c5_d_$r 150 python bench.py $B; line "cfg5 bdp reads, convert+write, issue run $r" c5_d_$r
done
run c5s2_p 150 python bench.py $B --heads 16 --kv-heads 16; line "cfg5 16h product" c5s2_p
FATTN_LIB=libfattn_deqfirst.so run c5s2_d 150 python bench.py $B --heads 16 --kv-heads 16; line "cfg5 16h dequant first" c5s2_d
cat $F/tests_tail.txt $F/ab.txt
