#!/bin/bash
# prefill phase stamps: lockstep vs ping-pong, Q8_0 and f16
source tools/gpu_round.sh
export TMPDIR=/tmp
run pfst1 120 python tools/pf_stamps.py --pipe 1
run pfst2 120 python tools/pf_stamps.py --pipe 2
run pfst3 120 python tools/pf_stamps.py --kv-type f16
run pfst4 120 python tools/pf_stamps.py --pipe 2 --no-mask
cat gpurun_out/pfst1.log gpurun_out/pfst2.log gpurun_out/pfst3.log gpurun_out/pfst4.log | grep -v amdgpu.ids
