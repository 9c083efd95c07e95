#!/bin/bash
# Round 3: config-3 planner sweep after the cheaper last-arriver merge:
# waves per workgroup x steps per wave x steps in flight (kernel time, HIP events).
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3s}
mkdir -p gpurun_out/$D
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --warmup 20"
for cfg in "8 2 1" "8 2 2" "8 1 1" "16 1 1" "4 4 2" "4 2 2" "8 3 1" "16 2 1" "8 4 1" "4 1 1"; do
  set -- $cfg
  n=w$1_s$2_i$3
  run $n 120 python bench.py $B --waves $1 --spw $2 --inflight $3
  echo "cfg3 waves=$1 spw=$2 inflight=$3 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$n.log) $(grep -o '"kernel": "[^"]*' gpurun_out/$n.log | head -1)" >> gpurun_out/$D/sweep.txt
done
run w8_s2_i1_again 120 python bench.py $B
echo "cfg3 planner (again) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/w8_s2_i1_again.log)" >> gpurun_out/$D/sweep.txt
cat gpurun_out/$D/sweep.txt
