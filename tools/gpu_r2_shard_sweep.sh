#!/bin/bash
# Config-5 per-GPU shard (4 heads, n_q = 64, N = 4096, Q8_0): planner sweep of
# KV chunk x waves x merge form, kernel-only bench lines into gpurun_out/shard/.
source tools/gpu_round.sh
mkdir -p gpurun_out/shard
B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --workload config5 --heads 4 --kv-heads 4 --steps 200 --warmup 20"
run planner 120 $B
grep '^{' gpurun_out/planner.log > gpurun_out/shard/planner.json || true
for c in 128 256 512 1024; do
  for w in 4 8; do
    for m in "" "--fused-merge"; do
      n=c${c}_w${w}${m:+_fused}
      run $n 120 $B --kv-chunk $c --waves $w $m
      grep '^{' gpurun_out/$n.log > gpurun_out/shard/$n.json || true
    done
  done
done
run mq 120 $B --pf 0 --kv-chunk 0
ls gpurun_out/shard | wc -l
