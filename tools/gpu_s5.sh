#!/bin/bash
# tagged hand-off: parity, then geometry sweep tagged vs counters
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
: > gpurun_out/tag_summary.txt
for g in "4 2" "2 2" "1 1"; do set -- $g
  for c in c3 c4; do
    X=""; [ $c = c4 ] && X="$C4"
    for t in "" "--untagged"; do
      out=$(timeout -k 10 60 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --spw $1 --inflight $2 $t $X 2>/dev/null | grep '^{')
      rc=$?; [ $rc -ne 0 ] && { echo "FAIL $c $g $t rc=$rc" >> gpurun_out/tag_summary.txt; exit 1; }
      python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('%s spw=%s inf=%s %-10s %7.2f us' % ('$c','$1','$2','$t', r['kernel_ms_avg']*1e3))" "$out" >> gpurun_out/tag_summary.txt
    done
  done
done
cat gpurun_out/tag_summary.txt
