#!/bin/bash
# Round 3: prefill kernel -- parity (pf tests), then the prefill shape with the
# four masks (zero per SURVEY §8d, random, causal, none) for Q8_0 and f16 K/V.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3pf}
mkdir -p gpurun_out/$D
run pytest_pf 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "pf"
B="--no-cpu-baseline --no-scale-ref --no-copy-peak --steps 5 --warmup 2"
for kv in q8_0 f16; do
  for m in zero random causal none; do
    run pf_${kv}_$m 180 python bench.py $B --prefill-kv $kv --prefill-mask $m
    grep -o '"prefill": {[^}]*}[^}]*}' gpurun_out/pf_${kv}_$m.log >> gpurun_out/$D/summary.txt || true
  done
done
cat gpurun_out/$D/summary.txt
