#!/bin/bash
# diagnostic-build breakdown of the split kernel (config 3 and 4) at several geometries
source tools/gpu_round.sh
export TMPDIR=/tmp
C4="--kv-type q4_0 --kv-heads 8 --kv-len 8192"
: > gpurun_out/diag_summary.txt
for lib in libfattn.so libfattn_nc.so libfattn_nctail.so libfattn_notail.so libfattn_nopub.so libfattn_noatomic.so libfattn_nomem.so libfattn_nomem_notail.so libfattn_nt.so; do
  for g in "4 2" "1 1" "2 2"; do set -- $g
    for c in c3 c4; do
      X=""; [ $c = c4 ] && X="$C4"
      out=$(FATTN_LIB=$lib timeout -k 10 60 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --spw $1 --inflight $2 $X 2>/dev/null | grep '^{')
      rc=$?
      [ $rc -ne 0 ] && { echo "FAIL $lib $c $g rc=$rc" >> gpurun_out/diag_summary.txt; [ $rc -ge 124 ] && exit $rc; continue; }
      python3 -c "import json,sys; r=json.loads(sys.argv[1]); print('%-26s %s spw=%s inf=%s  %7.2f us' % ('$lib','$c','$1','$2', r['kernel_ms_avg']*1e3))" "$out" >> gpurun_out/diag_summary.txt
    done
  done
done
cat gpurun_out/diag_summary.txt
