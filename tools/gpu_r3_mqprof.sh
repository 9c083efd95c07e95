#!/bin/bash
# Round 3: where config 5's time goes -- rocprofv3 kernel-trace stats of the
# multi-query and split plans (attention kernel vs merge kernel), and a
# KV-chunk sweep of the multi-query plan.
source tools/gpu_round.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/r3prof
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 50 --warmup 5"
for c in full shard; do
  X=""; [ $c = shard ] && X="--heads 4 --kv-heads 4"
  run kt_${c}_mq 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3prof/${c}_mq -o k -- python3 bench.py $N --workload config5 $X
  run kt_${c}_split 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3prof/${c}_split -o k -- python3 bench.py $N --workload config5 $X --no-mq
done
for ch in 128 512 1024 2048; do
  run full_mq_c$ch 120 python bench.py $N --workload config5 --kv-chunk $ch
done
for ch in 256 512 1024; do
  run shard_mq_c$ch 120 python bench.py $N --workload config5 --heads 4 --kv-heads 4 --kv-chunk $ch
done
for f in gpurun_out/full_mq_c*.log gpurun_out/shard_mq_c*.log; do echo "$f $(grep -o '"kernel_ms_avg": [0-9.]*' $f) $(grep -o 'grid([0-9,]*)' $f | head -1)"; done > gpurun_out/r3prof/chunk_sweep.txt
find gpurun_out/r3prof -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-8 "$f" | head -8; done > gpurun_out/r3prof/stats_summary.txt
cat gpurun_out/r3prof/chunk_sweep.txt gpurun_out/r3prof/stats_summary.txt
