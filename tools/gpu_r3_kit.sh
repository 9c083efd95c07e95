#!/bin/bash
# Round 3: last-arriver row merge with as few load slots as the chunk count
# needs (merge_row_parts<D, 4> for config 3's 8 chunks) -- tests, a same-box
# A/B against the previous library (FATTN_LIB=libfattn_prev.so), and the
# config-3 traffic / kernel-trace passes of the new library.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3k}
F=gpurun_out/$D
mkdir -p $F
run t_kit 600 python -u -m pytest tests/test_rehearsal.py tests/test_gpu_extra.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "rehearsal or row_merge or bd_chunk_merge or workspace or config3 or handoff_stress or determinis"
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --warmup 20"
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/$2.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$2.log)" >> $F/ab.txt; }
for r in 1 2 3; do
  FATTN_LIB=libfattn_prev.so run c3_prev_$r 120 python bench.py $B; line "cfg3 prev (merge_row_parts<128,16>) run $r" c3_prev_$r
  run c3_kit_$r 120 python bench.py $B; line "cfg3 kit (merge_row_parts<128,4>) run $r" c3_kit_$r
done
FATTN_LIB=libfattn_prev.so run c2_prev 120 python bench.py $B --kv-type f16 --kv-len 2048; line "cfg2 prev" c2_prev
run c2_kit 120 python bench.py $B --kv-type f16 --kv-len 2048; line "cfg2 kit" c2_kit
D2="--no-cpu-baseline --no-scale-ref --no-copy-peak --no-prefill --steps 50 --warmup 5"
run fetch_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/prof5_fetch -o f -- python3 bench.py $D2
run write_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/prof5_write -o w -- python3 bench.py $D2
python tools/pmc_summary.py --kernel fattn_split_kernel --traffic $F/traffic_r03_cfg3.json --bench-line gpurun_out/fetch_cfg3.log \
  $(find gpurun_out/prof5_fetch gpurun_out/prof5_write -name "*counter_collection.csv") > $F/traffic_cfg3.txt 2>&1
run kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5_kt -o kt -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
for f in $(find gpurun_out/prof5_kt -name "*kernel_stats.csv"); do cp "$f" $F/kernel_stats.csv; done
python tools/kstats.py $F/kernel_stats.csv > $F/kernel_stats_summary.txt
grep '^{' gpurun_out/kt.log > $F/bench_under_rocprof.json || true
grep -E "passed|failed" gpurun_out/t_kit.log | tail -2 > $F/tests_tail.txt
cat $F/ab.txt $F/tests_tail.txt $F/traffic_cfg3.txt $F/kernel_stats_summary.txt
