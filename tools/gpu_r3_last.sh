#!/bin/bash
# Round 3, last check of the committed tree: smoke, the default bench line,
# the two-rank rehearsal tests and the chunk-merge tests.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/final6
mkdir -p $F
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run tests 600 python -u -m pytest tests/test_rehearsal.py tests/test_gpu_extra.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "rehearsal or merge or workspace or config3 or golden"
run bench 600 python bench.py
grep '^{' gpurun_out/bench.log > $F/bench.json || true
grep -E "passed|failed" gpurun_out/tests.log | tail -2 > $F/tests_tail.txt
tail -2 gpurun_out/smoke.log > $F/smoke.txt
cat $F/smoke.txt $F/tests_tail.txt; python -c "import json; d=json.load(open('$F/bench.json')); print(d['value'], d['kernel_ms_avg'], d['roofline']['frac'], d['roofline']['traffic'], d['prefill']['roofline']['frac'])"
