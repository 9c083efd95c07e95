#!/bin/bash
# Same-box A/B: prefill with the next tile's dequantisation interleaved into
# the second P.V chain (libfattn_diag_pf_dqpv.so) against the product.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3ab2}
mkdir -p gpurun_out/$D
run pf_test 300 env FATTN_LIB=libfattn_diag_pf_dqpv.so python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "pf"
B="--no-cpu-baseline --no-scale-ref --no-copy-peak --steps 5 --warmup 2"
for rep in 1 2; do
  for lib in libfattn.so libfattn_diag_pf_dqpv.so; do
    for m in none zero; do
      n=pf_${lib%.so}_${m}_$rep
      FATTN_LIB=$lib run $n 180 python bench.py $B --prefill-mask $m
      echo "$n $(grep -o '"prefill": {[^}]*"kernel_ms_avg": [0-9.]*' gpurun_out/$n.log | grep -o '"kernel_ms_avg": [0-9.]*')" >> gpurun_out/$D/prefill_ab.txt
    done
  done
done
tail -2 gpurun_out/pf_test.log >> gpurun_out/$D/prefill_ab.txt
cat gpurun_out/$D/prefill_ab.txt
