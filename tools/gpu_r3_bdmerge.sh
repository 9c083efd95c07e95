#!/bin/bash
# Round 3: in-kernel chunk merge of multi-row tiles (batched-decode kernel and
# split kernel with 4+ chunks) -- parity first (merge forms, workspace garbage,
# graph replays, config-5 parity), then same-box A/Bs, in-kernel vs second
# launch: config 5 (32 heads, bd), its 2-rank shard (16 heads, bd), its 8-rank
# shard (4 heads, split), config 4 (split); and config 3 (unchanged path).
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3m}
mkdir -p gpurun_out/$D
run t_merge 500 python -u -m pytest tests/test_gpu_extra.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "merge or workspace or replay or graph or config5 or config4 or bd"
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --warmup 20"
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/$2.log) $(grep -o '"kernel": "[^"]*' gpurun_out/$2.log | head -1)" >> gpurun_out/$D/ab.txt; }
for r in 1 2; do
  for m in 0 1; do
    run c5_m${m}_$r 120 python bench.py $B --workload config5 --merge-in-kernel $((1 - m)); line "cfg5 h32 merge_launch=$m run $r" c5_m${m}_$r
    run c5s8_m${m}_$r 120 python bench.py $B --workload config5 --heads 4 --kv-heads 4 --merge-in-kernel $((1 - m)); line "cfg5 h4 merge_launch=$m run $r" c5s8_m${m}_$r
    run c4_m${m}_$r 120 python bench.py $B --kv-type q4_0 --kv-heads 8 --kv-len 8192 --merge-in-kernel $((1 - m)); line "cfg4 merge_launch=$m run $r" c4_m${m}_$r
  done
done
for m in 0 1; do
  run c5h16_m$m 120 python bench.py $B --workload config5 --heads 16 --kv-heads 16 --merge-in-kernel $((1 - m)); line "cfg5 h16 merge_launch=$m" c5h16_m$m
done
run c3 120 python bench.py $B; line "cfg3" c3
tail -3 gpurun_out/t_merge.log > gpurun_out/$D/tests_tail.txt
grep -E "PASSED|FAILED|ERROR" gpurun_out/t_merge.log | tail -80 >> gpurun_out/$D/tests_tail.txt
cat gpurun_out/$D/ab.txt gpurun_out/$D/tests_tail.txt
