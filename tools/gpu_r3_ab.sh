#!/bin/bash
# Round 3 same-box A/Bs: (1) prefill zero-mask tiles with / without the
# skipped mask wait + reads (product vs libfattn_diag_pf_nozero.so), three
# alternating runs each; (2) config-5 shards of 4 / 8 / 16 / 32 heads on the
# split kernel (--no-mq) against the batched-decode kernel (--bd 2) and the
# planner's pick.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3ab}
mkdir -p gpurun_out/$D
B="--no-cpu-baseline --no-scale-ref --no-copy-peak --steps 5 --warmup 2"
for rep in 1 2 3; do
  for lib in libfattn.so libfattn_diag_pf_nozero.so; do
    for m in zero causal; do
      n=pf_${lib%.so}_${m}_$rep
      FATTN_LIB=$lib run $n 180 python bench.py $B --prefill-mask $m
      echo "$n $(grep -o '"prefill": {[^}]*"kernel_ms_avg": [0-9.]*' gpurun_out/$n.log | grep -o '"kernel_ms_avg": [0-9.]*')" >> gpurun_out/$D/prefill_ab.txt
    done
  done
done
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
for h in 4 8 16 32; do
  for v in "auto:" "split:--no-mq" "bd:--bd 2"; do
    name=${v%%:*}; opt=${v#*:}
    n=c5_h${h}_$name
    run $n 120 python bench.py $N --heads $h --kv-heads $h $opt
    echo "$n $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$n.log) $(grep -o '"kernel": "[^"]*' gpurun_out/$n.log | head -1 | cut -c1-60)" >> gpurun_out/$D/config5_heads.txt
  done
done
cat gpurun_out/$D/prefill_ab.txt gpurun_out/$D/config5_heads.txt
