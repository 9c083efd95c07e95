#!/bin/bash
# Round-end evidence: GPU suite, smoke, the default bench line, the rocprofv3
# kernel-trace summary of the bench, and the PMC passes (one per block budget:
# FETCH_SIZE, WRITE_SIZE, the prefill MFMA counters).  Copies the CSVs to
# gpurun_out/final/ under fixed names.
source tools/gpu_round.sh
export TMPDIR=/tmp
mkdir -p gpurun_out/final
[ -n "$PROF_ONLY" ] || run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread
[ -n "$PROF_ONLY" ] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
if [ -z "$PROF_ONLY" ]; then
  run bench 600 python bench.py
  grep '^{' gpurun_out/bench.log > gpurun_out/final/bench.json || true
fi
run kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
D="--no-cpu-baseline --no-scale-ref --no-copy-peak"
run pmc_fetch 180 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o f -- python3 bench.py --steps 50 --warmup 5 --no-prefill $D
run pmc_write 180 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/prof_write -o w -- python3 bench.py --steps 50 --warmup 5 --no-prefill $D
run pmc_mfma 300 rocprofv3 --output-format csv --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/prof_mfma -o m -- python3 bench.py --steps 5 --warmup 2 $D
run pmc_coexec 300 rocprofv3 --output-format csv --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/prof_coexec -o c -- python3 bench.py --steps 5 --warmup 2 $D
for d in kt fetch write mfma coexec; do
  for f in $(find gpurun_out/prof_$d -name "*.csv"); do cp "$f" "gpurun_out/final/${d}_$(basename $f | sed 's/^[0-9]*_//')"; done
done
ls -la gpurun_out/final
