#!/bin/bash
# Run-to-run spread on one box: the default bench line three times (config 3),
# then one line per BASELINE.json config 2/4/5 (5 = the 4-head per-GPU shard
# and all 32 heads), kernel-only legs.  Lines land in gpurun_out/spread/.
source tools/gpu_round.sh
mkdir -p gpurun_out/spread
N="--no-cpu-baseline --no-prefill --no-scale-ref"
for i in 1 2 3; do
  run cfg3_run$i 180 python bench.py $N
  grep '^{' gpurun_out/cfg3_run$i.log > gpurun_out/spread/cfg3_run$i.json || true
done
run cfg2 180 python bench.py $N --kv-type f16 --kv-len 2048
run cfg4 180 python bench.py $N --kv-type q4_0 --kv-heads 8 --kv-len 8192
run cfg5_shard 180 python bench.py $N --workload config5 --heads 4 --kv-heads 4
run cfg5_full 180 python bench.py $N --workload config5
for s in cfg2 cfg4 cfg5_shard cfg5_full; do grep '^{' gpurun_out/$s.log > gpurun_out/spread/$s.json || true; done
ls -la gpurun_out/spread
