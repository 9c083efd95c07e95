#!/bin/bash
# Round 3: one-row hand-off forms -- parity first (new cases, workspace and
# stress tests), then a same-box A/B of config 3 and config 2 (granules vs drain).
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3h}
mkdir -p gpurun_out/$D
run t_handoff 400 python -u -m pytest tests/test_gpu_extra.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "handoff or workspace or graph or determinis"
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --warmup 20"
for r in 1 2 3; do
  for h in 0 1; do
    run c3_h${h}_$r 120 python bench.py $B --handoff $h
    echo "cfg3 handoff=$h run $r $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/c3_h${h}_$r.log) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/c3_h${h}_$r.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c3_h${h}_$r.log)" >> gpurun_out/$D/ab.txt
  done
done
for h in 0 1; do
  run c2_h$h 120 python bench.py $B --handoff $h --kv-type f16 --kv-len 2048
  echo "cfg2 handoff=$h $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/c2_h$h.log) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/c2_h$h.log)" >> gpurun_out/$D/ab.txt
done
grep -h "kernel\"" gpurun_out/c3_h0_1.log | head -2 > /dev/null
tail -3 gpurun_out/t_handoff.log > gpurun_out/$D/tests_tail.txt
cat gpurun_out/$D/ab.txt gpurun_out/$D/tests_tail.txt
