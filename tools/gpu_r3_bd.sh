#!/bin/bash
# Round 3: the batched-decode kernel (fattn_bd.h) -- parity, then config 5
# (all 32 heads; the 4-head per-GPU shard) with a KV-chunk sweep, kernel-trace
# stats for the attention and merge kernels.
source tools/gpu_round.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/r3bd
run pytest_bd 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bd or config5 or mq"
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10"
run cfg5_full 120 python bench.py $N --workload config5
run cfg5_shard 120 python bench.py $N --workload config5 --heads 4 --kv-heads 4
for ch in 256 1024; do run full_c$ch 120 python bench.py $N --workload config5 --kv-chunk $ch; done
for ch in 256 512 1024; do run shard_c$ch 120 python bench.py $N --workload config5 --heads 4 --kv-heads 4 --kv-chunk $ch; done
run kt_full 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3bd/kt_full -o k -- python3 bench.py $N --workload config5
run kt_shard 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3bd/kt_shard -o k -- python3 bench.py $N --workload config5 --heads 4 --kv-heads 4
for f in gpurun_out/cfg5_*.log gpurun_out/full_c*.log gpurun_out/shard_c*.log; do echo "$f $(grep -o '"kernel_ms_avg": [0-9.]*' $f) $(grep -o 'grid([0-9,]*)' $f | head -1)"; done > gpurun_out/r3bd/summary.txt
python tools/kstats.py $(find gpurun_out/r3bd -name "*kernel_stats.csv" | sort) >> gpurun_out/r3bd/summary.txt
cat gpurun_out/r3bd/summary.txt
