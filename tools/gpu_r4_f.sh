#!/bin/bash
# Round 4: XCD-grouped workgroup order for the batched-decode kernels
# (--bd-xcd 2) against the plain order (--bd-xcd 1): time and HBM traffic
# (FETCH_SIZE / WRITE_SIZE) on config 5, its 2-rank shard; the role form at head
# dim 96 against the planner's previous pick (split kernel); their tests and
# the prefill tests at head dims 80 (f16) and 96.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4f
mkdir -p $F
run t_bd 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "bdp or bd_ or xcd or pf_d80 or pf_d96"
grep -E "passed|failed" gpurun_out/t_bd.log | tail -2 > $F/tests_tail.txt
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5"
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1) $(grep -o '"kernel_ms_median": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
for r in 1 2; do
  run c5_x2_$r 200 python bench.py $B --bd-xcd 2; line "cfg5 32h bdp xcd-grouped run $r" c5_x2_$r
  run c5_x1_$r 200 python bench.py $B --bd-xcd 1; line "cfg5 32h bdp plain order run $r" c5_x1_$r
done
run c5s2_x2 200 python bench.py $B --heads 16 --kv-heads 16 --bd-xcd 2; line "cfg5 16h bdp xcd-grouped" c5s2_x2
run c5s2_x1 200 python bench.py $B --heads 16 --kv-heads 16 --bd-xcd 1; line "cfg5 16h bdp plain order" c5s2_x1
run c5d96_bdp 200 python bench.py $B --head-dim 96; line "cfg5-shape D96 bdp" c5d96_bdp
run c5d96_split 200 python bench.py $B --head-dim 96 --bd 1 --no-mq; line "cfg5-shape D96 split (bd off)" c5d96_split
D="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5 --workload config5"
for x in 1 2; do
  run fetch_x$x 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r4f_f$x -o f -- python3 bench.py $D --bd-xcd $x
  run write_x$x 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r4f_w$x -o w -- python3 bench.py $D --bd-xcd $x
  python tools/pmc_summary.py --kernel fattn_bdp_kernel --traffic $F/traffic_cfg5_x$x.json --bench-line gpurun_out/fetch_x$x.log \
    $(find gpurun_out/r4f_f$x gpurun_out/r4f_w$x -name "*counter_collection.csv") > $F/traffic_cfg5_x$x.txt 2>&1
done
cat $F/tests_tail.txt $F/ab.txt $F/traffic_cfg5_x1.txt $F/traffic_cfg5_x2.txt
