#!/bin/bash
# Same-box A/B: prefill raw-tile DMA issued behind the S^T chains, K operand
# reads split, stagger path removed (product) against
# the previous form (libfattn_diag_pf_oldwait.so); prefill parity first.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3ab4}
mkdir -p gpurun_out/$D
run pf_test 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "pf"
B="--no-cpu-baseline --no-scale-ref --no-copy-peak --steps 5 --warmup 2"
for rep in 1 2 3; do
  for lib in libfattn.so libfattn_diag_pf_oldwait.so; do
    for kv in q8_0 f16; do
      n=pf_${lib%.so}_${kv}_$rep
      FATTN_LIB=$lib run $n 180 python bench.py $B --prefill-kv $kv
      echo "$n $(grep -o '"prefill": {[^}]*"kernel_ms_avg": [0-9.]*' gpurun_out/$n.log | grep -o '"kernel_ms_avg": [0-9.]*')" >> gpurun_out/$D/prefill_ab.txt
    done
  done
done
tail -2 gpurun_out/pf_test.log >> gpurun_out/$D/prefill_ab.txt
cat gpurun_out/$D/prefill_ab.txt
