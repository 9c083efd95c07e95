#!/bin/bash
# Round 4: config 4 (Q4_0, 32 q / 8 kv heads, N = 8192, one query) planner
# sweep -- KV chunk (32 / 16 / 8 chunks per head) x waves per workgroup x merge
# form (second launch / last-arriving workgroup) -- and its kernel-trace split.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4g
mkdir -p $F
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --heads 32 --kv-heads 8 --kv-len 8192 --kv-type q4_0"
line() { echo "$1 $(grep -o '"kernel": "[^"]*"' gpurun_out/$2.log | head -1) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/sweep.txt; }
run c4_pl 200 python bench.py $B; line "cfg4 planner" c4_pl
for ch in 256 512 1024; do
  for w in 4 8; do
    run c4_${ch}_$w 200 python bench.py $B --kv-chunk $ch --waves $w; line "cfg4 chunk $ch waves $w" c4_${ch}_$w
    run c4_${ch}_${w}_f 200 python bench.py $B --kv-chunk $ch --waves $w --fused-merge; line "cfg4 chunk $ch waves $w fused merge" c4_${ch}_${w}_f
  done
done
run kt4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4g_kt -o kt -- python3 bench.py $B
for f in $(find gpurun_out/r4g_kt -name "*kernel_stats.csv"); do cp "$f" $F/kernel_stats_cfg4.csv; done
python tools/kstats.py $F/kernel_stats_cfg4.csv > $F/kernel_stats_cfg4.txt 2>&1
cat $F/sweep.txt $F/kernel_stats_cfg4.txt
