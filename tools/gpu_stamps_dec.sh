#!/bin/bash
# fattn_dec_kernel phase stamps (diagnostic library) on configs 2-4, plus the new bench line
source tools/gpu_round.sh
export TMPDIR=/tmp
run t_wm 120 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 60 --timeout-method thread -k "wave_merge"
for v in "" "--diag 1" "--diag 2" "--dec-compute 8"; do
  run st_c3 60 python tools/dec_stamps.py $v; cat gpurun_out/st_c3.log >> gpurun_out/stamps.txt
done
run st_c2 60 python tools/dec_stamps.py --kv-type f16 --kv-len 2048; cat gpurun_out/st_c2.log >> gpurun_out/stamps.txt
run st_c4 60 python tools/dec_stamps.py --kv-type q4_0 --kv-heads 8 --kv-len 8192; cat gpurun_out/st_c4.log >> gpurun_out/stamps.txt
run bench1 200 python bench.py --no-prefill --cpu-seconds 4
cat gpurun_out/stamps.txt
