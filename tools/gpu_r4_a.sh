#!/bin/bash
# Round 4, first box: the whole GPU suite (the chunk merges now read their
# partials through compiler-tracked sc1 buffer loads; the N>1 value line is the
# config-5 head shard with one gather per timed step, rehearsed on one GPU),
# smoke, and the default N=1 bench line.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4a
mkdir -p $F
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run t_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 250 --timeout-method thread
run bench 600 python bench.py --steps 100 --warmup 10
grep '^{' gpurun_out/bench.log > $F/bench.json || true
grep -E "passed|failed" gpurun_out/t_all.log | tail -2 > $F/tests_tail.txt
cat $F/tests_tail.txt
