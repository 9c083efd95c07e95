#!/bin/bash
source tools/gpu_round.sh
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run harness_q8 120 ggml-cuda-experiments_amd/bin/kernel_test --kv-size 4096 --kv-type q8_0 --heads 32 --kv-heads 32
run harness_f16 120 ggml-cuda-experiments_amd/bin/kernel_test
run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
run bench 400 python bench.py --steps 100 --warmup 10 --cpu-seconds 3
