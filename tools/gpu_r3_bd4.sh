#!/bin/bash
# Round 3: batched-decode kernel iteration: parity subset, config 5 full and
# shard (bench + kernel-trace), phase stamps (diagnostic library).
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3bd4}
mkdir -p gpurun_out/$D
run pytest_bd 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bd or config5 or shard"
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10"
run kt_full 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/kt_full -o k -- python3 bench.py $N --workload config5
run kt_shard 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/kt_shard -o k -- python3 bench.py $N --workload config5 --heads 4 --kv-heads 4
run st_shard 120 python tools/stamps_bd.py --heads 4
run st_full 120 python tools/stamps_bd.py --heads 32
for f in gpurun_out/kt_full.log gpurun_out/kt_shard.log; do echo "$f $(grep -o '"kernel_ms_avg": [0-9.]*' $f) $(grep -o 'grid([0-9,]*)' $f | head -1)"; done > gpurun_out/$D/summary.txt
python tools/kstats.py $(find gpurun_out/$D -name "*kernel_stats.csv" | sort) >> gpurun_out/$D/summary.txt
cp gpurun_out/st_shard.log gpurun_out/st_full.log gpurun_out/$D/
cat gpurun_out/$D/summary.txt
