#!/bin/bash
# Round 3: whole GPU suite, the prefill shape with the four masks, config 5
# full / shard kernel traces.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3c}
mkdir -p gpurun_out/$D
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
B="--no-cpu-baseline --no-scale-ref --no-copy-peak --steps 5 --warmup 2"
for kv in q8_0 f16; do
  for m in zero random causal none; do
    run pf_${kv}_$m 180 python bench.py $B --prefill-kv $kv --prefill-mask $m
    grep -o '"prefill": {[^}]*}[^}]*}' gpurun_out/pf_${kv}_$m.log >> gpurun_out/$D/prefill.txt || true
  done
done
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10"
run kt_full 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/kt_full -o k -- python3 bench.py $N --workload config5
run kt_shard 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/kt_shard -o k -- python3 bench.py $N --workload config5 --heads 4 --kv-heads 4
run kt_shard2 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/kt_shard2 -o k -- python3 bench.py $N --workload config5 --heads 16 --kv-heads 16
for f in gpurun_out/kt_full.log gpurun_out/kt_shard.log gpurun_out/kt_shard2.log; do echo "$f $(grep -o '"kernel_ms_avg": [0-9.]*' $f) $(grep -o 'grid([0-9,]*)' $f | head -1)"; done > gpurun_out/$D/summary.txt
python tools/kstats.py $(find gpurun_out/$D -name "*kernel_stats.csv" | sort) >> gpurun_out/$D/summary.txt
tail -3 gpurun_out/pytest_gpu.log >> gpurun_out/$D/summary.txt
cat gpurun_out/$D/prefill.txt gpurun_out/$D/summary.txt
