#!/bin/bash
# Round 3, step 1: the multi-query kernel with the second-launch merge on
# config 5 (one GPU: all 32 heads; the 4-head per-GPU shard), against the split
# kernel (--no-mq); parity of the mq / config-5 tests and the 2-rank rehearsal.
source tools/gpu_round.sh
mkdir -p gpurun_out/r3mq
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak"
run pytest_mq 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "mq or config5"
run rehearse 300 python -u -m pytest tests/test_rehearsal.py -m gpu -x -q -s -p no:cacheprovider --timeout 280 --timeout-method thread
run cfg5_full_mq 180 python bench.py $N --workload config5
run cfg5_full_split 180 python bench.py $N --workload config5 --no-mq
run cfg5_shard_mq 180 python bench.py $N --workload config5 --heads 4 --kv-heads 4
run cfg5_shard_split 180 python bench.py $N --workload config5 --heads 4 --kv-heads 4 --no-mq
run cfg3 300 python bench.py --no-scale-ref
for s in cfg5_full_mq cfg5_full_split cfg5_shard_mq cfg5_shard_split cfg3; do grep '^{' gpurun_out/$s.log > gpurun_out/r3mq/$s.json || true; done
grep '^{' gpurun_out/rehearse.log > gpurun_out/r3mq/rehearse.json || true
