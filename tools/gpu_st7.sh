#!/bin/bash
# decode phase timeline after the K/mask-first change (configs 3 and 4)
source tools/gpu_round.sh
export TMPDIR=/tmp
run st7_c3 120 python tools/stamps.py
run st7_c4 120 python tools/stamps.py --kv-type q4_0 --kv-heads 8 --kv-len 8192
cat gpurun_out/st7_c3.log gpurun_out/st7_c4.log | grep -v amdgpu.ids
