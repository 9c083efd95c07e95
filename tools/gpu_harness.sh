#!/bin/bash
# the kernel_test harness (src/kernel_test.h counterpart) and smoke() on the final tree
source tools/gpu_round.sh
export TMPDIR=/tmp
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
run kt_f16 60 ggml-cuda-experiments_amd/bin/kernel_test
run kt_f16_ext 60 ggml-cuda-experiments_amd/bin/kernel_test --no-kv-parallel
run kt_q8 60 ggml-cuda-experiments_amd/bin/kernel_test --kv-type q8_0 --kv-size 4096 --heads 32 --kv-heads 32
run kt_q4_256 60 ggml-cuda-experiments_amd/bin/kernel_test --kv-type q4_0 --kv-size 8192 --head-dim 256
tail -n 4 gpurun_out/smoke.log gpurun_out/kt_*.log
