#!/bin/bash
# Round 4, first box: the whole GPU suite (chunk merges through compiler-tracked
# sc1 loads; the f16 batched-decode path; the N>1 value line = config-5 head
# shard with one gather per timed step, rehearsed on one GPU), smoke, the
# default N=1 bench line, and config 5's shape over f16 K/V: batched-decode
# kernel vs the split kernel it replaces.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4a
mkdir -p $F
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run t_all 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread
run bench 600 python bench.py --steps 100 --warmup 10
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10 --workload config5 --kv-type f16"
run c5f16_bd 300 python bench.py $B
run c5f16_split 300 python bench.py $B --bd 1
grep '^{' gpurun_out/bench.log > $F/bench.json || true
for n in c5f16_bd c5f16_split; do echo "$n $(grep -o '"kernel": "[^"]*"' gpurun_out/$n.log) $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$n.log)" >> $F/c5f16.txt; done
grep -E "passed|failed" gpurun_out/t_all.log | tail -2 > $F/tests_tail.txt
cat $F/tests_tail.txt $F/c5f16.txt
