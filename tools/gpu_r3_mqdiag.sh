#!/bin/bash
# Multi-query kernel phase costs on config 5 (full and shard): the product
# library against diagnostic builds without memory / dequant / compute.
source tools/gpu_round.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/r3diag; D=${DIAGDIR:-r3diag}
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 50 --warmup 5"
for lib in libfattn.so libfattn_diag_mq_nomem.so libfattn_diag_mq_nodeq.so libfattn_diag_mq_nocompute.so libfattn_diag_mq_dmaonly.so; do
  for c in full shard; do
    X=""; [ $c = shard ] && X="--heads 4 --kv-heads 4"
    n=${lib%.so}_$c
    FATTN_LIB=$lib run kt_$n 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/$n -o k -- python3 bench.py $N --workload config5 $X
  done
done
for f in $(find gpurun_out/$D -name "*kernel_stats.csv" | sort); do :; done; python tools/kstats.py $(find gpurun_out/$D -name "*kernel_stats.csv" | sort) > gpurun_out/$D/summary.txt
cat gpurun_out/$D/summary.txt
