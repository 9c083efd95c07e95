#!/bin/bash
# Round 4: the compute / build-role batched-decode kernel (fattn_bdp.h) --
# its parity tests, the batched-decode / ABI tests around it, then config 5
# (one GPU and the 2-rank shard's 16 heads) with the all-waves form (--bd 2)
# and the role form (--bd 3), alternating on one box.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4b
mkdir -p $F
run t_bdp 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py tests/test_abi.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bd or config5 or merge"
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
line() { echo "$1 $(grep -o '"kernel": "[^"]*"' gpurun_out/$2.log | head -1) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
for r in 1 2; do
  run c5_bd_$r 200 python bench.py $B --bd 2; line "cfg5 32 heads bd (all waves) run $r" c5_bd_$r
  run c5_bdp_$r 200 python bench.py $B --bd 3; line "cfg5 32 heads bdp (roles) run $r" c5_bdp_$r
  run c5s2_bd_$r 200 python bench.py $B --heads 16 --kv-heads 16 --bd 2; line "cfg5 16 heads bd run $r" c5s2_bd_$r
  run c5s2_bdp_$r 200 python bench.py $B --heads 16 --kv-heads 16 --bd 3; line "cfg5 16 heads bdp run $r" c5s2_bdp_$r
done
run c5q4_bd 200 python bench.py $B --kv-type q4_0 --bd 2; line "cfg5-shape q4_0 bd" c5q4_bd
run c5q4_bdp 200 python bench.py $B --kv-type q4_0 --bd 3; line "cfg5-shape q4_0 bdp" c5q4_bdp
grep -E "passed|failed" gpurun_out/t_bdp.log | tail -2 > $F/tests_tail.txt
cat $F/tests_tail.txt $F/ab.txt
# per-kernel durations (attention kernel vs the merge launch), both forms
run kt_bd 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_kt_bd -o kt -- python3 bench.py $B --bd 2
run kt_bdp 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b_kt_bdp -o kt -- python3 bench.py $B --bd 3
for f in $(find gpurun_out/r4b_kt_bd gpurun_out/r4b_kt_bdp -name "*kernel_stats.csv"); do echo "== $f"; python3 tools/kstats.py $f; done > $F/kstats.txt 2>&1
cat $F/kstats.txt
