#!/bin/bash
# Round 3: chunk merges reduce over the valid part lanes only (head_reduce) --
# the whole GPU suite, a same-box A/B against the previous library
# (FATTN_LIB=libfattn_prev.so), then the config-3 traffic passes and the default
# bench line of the new library.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3r}
F=gpurun_out/$D
mkdir -p $F
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --warmup 20"
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/$2.log)" >> $F/ab.txt; }
for r in 1 2 3; do
  FATTN_LIB=libfattn_prev.so run c3_prev_$r 120 python bench.py $B; line "cfg3 prev (64-lane reductions) run $r" c3_prev_$r
  run c3_red_$r 120 python bench.py $B; line "cfg3 head_reduce run $r" c3_red_$r
done
FATTN_LIB=libfattn_prev.so run c2_prev 120 python bench.py $B --kv-type f16 --kv-len 2048; line "cfg2 prev" c2_prev
run c2_red 120 python bench.py $B --kv-type f16 --kv-len 2048; line "cfg2 head_reduce" c2_red
FATTN_LIB=libfattn_prev.so run c4_prev 120 python bench.py $B --kv-type q4_0 --kv-heads 8 --kv-len 8192; line "cfg4 prev" c4_prev
run c4_red 120 python bench.py $B --kv-type q4_0 --kv-heads 8 --kv-len 8192; line "cfg4 head_reduce" c4_red
D2="--no-cpu-baseline --no-scale-ref --no-copy-peak --no-prefill --steps 50 --warmup 5"
run fetch_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/prof6_fetch -o f -- python3 bench.py $D2
run write_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/prof6_write -o w -- python3 bench.py $D2
python tools/pmc_summary.py --kernel fattn_split_kernel --traffic $F/traffic_r03_cfg3.json --bench-line gpurun_out/fetch_cfg3.log \
  $(find gpurun_out/prof6_fetch gpurun_out/prof6_write -name "*counter_collection.csv") > $F/traffic_cfg3.txt 2>&1
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3 > $F/pytest_gpu_tail.txt
cat $F/ab.txt $F/pytest_gpu_tail.txt $F/traffic_cfg3.txt
