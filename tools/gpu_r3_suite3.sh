#!/bin/bash
# Round 3: the whole GPU suite and smoke on the final tree, then the default bench line.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/final5
mkdir -p $F
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python bench.py
grep '^{' gpurun_out/bench.log > $F/bench.json || true
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3 > $F/pytest_gpu_tail.txt
tail -2 gpurun_out/smoke.log > $F/smoke.txt
cat $F/pytest_gpu_tail.txt $F/smoke.txt $F/bench.json
