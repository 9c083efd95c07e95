#!/bin/bash
# Round 4: prefill epilogue -- normalised rows parked in LDS and stored as whole
# rows (product) against the row-per-lane stores from the accumulator layout
# (libfattn_pfdirect.so): prefill tests, time (zero / random mask, f16) and
# WRITE_SIZE / FETCH_SIZE.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4h
mkdir -p $F
run t_pf 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_extra.py -m gpu -x -q -p no:cacheprovider \
  --timeout 250 --timeout-method thread -k "pf or prefill"
grep -E "passed|failed" gpurun_out/t_pf.log | tail -2 > $F/tests_tail.txt
line() { echo "$1 $(grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/$2.log | head -1)" >> $F/ab.txt; }
for r in 1 2; do
  run pf_rows_$r 150 python bench.py --prefill-only; line "prefill q8_0 zero mask, whole-row stores run $r" pf_rows_$r
  FATTN_LIB=libfattn_pfdirect.so run pf_dir_$r 150 python bench.py --prefill-only; line "prefill q8_0 zero mask, row-per-lane stores run $r" pf_dir_$r
  run pfr_rows_$r 150 python bench.py --prefill-only --prefill-mask random; line "prefill q8_0 random mask, whole-row stores run $r" pfr_rows_$r
  FATTN_LIB=libfattn_pfdirect.so run pfr_dir_$r 150 python bench.py --prefill-only --prefill-mask random; line "prefill q8_0 random mask, row-per-lane stores run $r" pfr_dir_$r
done
run pff_rows 150 python bench.py --prefill-only --prefill-kv f16 --prefill-mask none; line "prefill f16 no mask, whole-row stores" pff_rows
FATTN_LIB=libfattn_pfdirect.so run pff_dir 150 python bench.py --prefill-only --prefill-kv f16 --prefill-mask none; line "prefill f16 no mask, row-per-lane stores" pff_dir
run fetch_pf 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r4h_pfetch -o f -- python3 bench.py --prefill-only
run write_pf 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r4h_pwrite -o w -- python3 bench.py --prefill-only
python tools/pmc_summary.py --kernel fattn_pf_kernel --traffic $F/traffic_prefill_rows.json --bench-line gpurun_out/fetch_pf.log \
  $(find gpurun_out/r4h_pfetch gpurun_out/r4h_pwrite -name "*counter_collection.csv") > $F/traffic_prefill_rows.txt 2>&1
cat $F/tests_tail.txt $F/ab.txt $F/traffic_prefill_rows.txt
