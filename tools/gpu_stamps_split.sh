#!/bin/bash
# split kernel phase stamps (diagnostic library) on configs 3, 4, 2
source tools/gpu_round.sh
export TMPDIR=/tmp
run st3 60 python tools/stamps.py
run st4 60 python tools/stamps.py --kv-type q4_0 --kv-heads 8 --kv-len 8192
run st2 60 python tools/stamps.py --kv-type f16 --kv-len 2048
cat gpurun_out/st3.log gpurun_out/st4.log gpurun_out/st2.log
