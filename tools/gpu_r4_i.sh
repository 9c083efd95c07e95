#!/bin/bash
# Round 4: prefill, quantised K/V -- the raw words of tile s + 1 read before
# tile s's S^T operand reads and converted after its S^T chains (product)
# against reads + conversion + image writes in one piece before the compute
# (libfattn_deqinl.so, FATTN_PF_DEQ_INLINE): prefill tests, time.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4i
mkdir -p $F
run t_pf 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "pf or prefill"
grep -E "passed|failed" gpurun_out/t_pf.log | tail -2 > $F/tests_tail.txt
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
for r in 1 2 3; do
  run pf_new_$r 150 python bench.py --prefill-only; line "prefill q8_0 zero mask, early raw reads run $r" pf_new_$r
  FATTN_LIB=libfattn_deqinl.so run pf_old_$r 150 python bench.py --prefill-only; line "prefill q8_0 zero mask, inline dequant run $r" pf_old_$r
done
for r in 1 2; do
  run pfr_new_$r 150 python bench.py --prefill-only --prefill-mask random; line "prefill q8_0 random mask, early raw reads run $r" pfr_new_$r
  FATTN_LIB=libfattn_deqinl.so run pfr_old_$r 150 python bench.py --prefill-only --prefill-mask random; line "prefill q8_0 random mask, inline dequant run $r" pfr_old_$r
  run pfq4_new_$r 150 python bench.py --prefill-only --prefill-kv q4_0; line "prefill q4_0 zero mask, early raw reads run $r" pfq4_new_$r
  FATTN_LIB=libfattn_deqinl.so run pfq4_old_$r 150 python bench.py --prefill-only --prefill-kv q4_0; line "prefill q4_0 zero mask, inline dequant run $r" pfq4_old_$r
done
# role-form batched decode: the build waves' raw reads before their DMA issue
# (product) against after it (libfattn_rdlate.so, FATTN_BDP_READ_LATE)
run t_bdp 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bdp"
grep -E "passed|failed" gpurun_out/t_bdp.log | tail -2 >> $F/tests_tail.txt
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
for r in 1 2 3; do
  run c5_early_$r 150 python bench.py $B; line "cfg5 bdp raw reads before the DMA issue run $r" c5_early_$r
  FATTN_LIB=libfattn_rdlate.so run c5_late_$r 150 python bench.py $B; line "cfg5 bdp raw reads after the DMA issue run $r" c5_late_$r
done
cat $F/tests_tail.txt $F/ab.txt
