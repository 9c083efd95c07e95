#!/bin/bash
# round-2 check: whole GPU suite, harness, the sharded bench path rehearsed on one GPU
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread
run rehearse2 300 env FATTN_BENCH_REHEARSE=1 python bench.py --gpus 2 --steps 50 --warmup 5
cat gpurun_out/rehearse2.log | grep '^{' || true
run bench1 300 python bench.py --no-prefill --cpu-seconds 4
