#!/bin/bash
# Round-4 evidence on a final tree (two calls): GPU suite and smoke; the default bench line,
# the two-rank rehearsal of the default N > 1 line (config-5 head shard, one
# gather per step), the rocprofv3 kernel-trace summary of the bench, and the
# FETCH_SIZE / WRITE_SIZE passes (traffic files tagged with plan + source hash)
# for config 3 and for the prefill shape (SURVEY's zero mask, as the bench's
# prefill object).  Summaries land in gpurun_out/r4final/.
#   PART=tests: the GPU suite and smoke only; PART=prof: everything else.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4final
mkdir -p $F
if [ "$PART" = tests ]; then
  run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
  run smoke 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  tail -3 gpurun_out/pytest_gpu.log > $F/pytest_gpu_tail.txt 2>/dev/null
  tail -2 gpurun_out/smoke.log > $F/smoke.txt 2>/dev/null
  cat $F/pytest_gpu_tail.txt $F/smoke.txt
  exit 0
fi
if [ -z "$PROF_ONLY" ]; then
  run bench 600 python bench.py
  grep '^{' gpurun_out/bench.log > $F/bench.json || true
  FATTN_BENCH_REHEARSE=1 run rehearse_head 300 python bench.py --gpus 2 --steps 20 --warmup 5
  grep '^{' gpurun_out/rehearse_head.log > $F/rehearse_world2_head.json || true
fi
run kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_kt -o kt -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
D="--no-cpu-baseline --no-scale-ref --no-copy-peak --no-prefill --steps 50 --warmup 5"
run fetch_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r4f_fetch -o f -- python3 bench.py $D
run write_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r4f_write -o w -- python3 bench.py $D
python tools/pmc_summary.py --kernel fattn_split_kernel --traffic $F/traffic_r04_cfg3.json --bench-line gpurun_out/fetch_cfg3.log \
  $(find gpurun_out/r4f_fetch gpurun_out/r4f_write -name "*counter_collection.csv") > $F/traffic_cfg3.txt 2>&1
run fetch_pf 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r4f_pfetch -o f -- python3 bench.py --prefill-only
run write_pf 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r4f_pwrite -o w -- python3 bench.py --prefill-only
python tools/pmc_summary.py --kernel fattn_pf_kernel --traffic $F/traffic_r04_prefill.json --bench-line gpurun_out/fetch_pf.log \
  $(find gpurun_out/r4f_pfetch gpurun_out/r4f_pwrite -name "*counter_collection.csv") > $F/traffic_prefill.txt 2>&1
# the prefill with its query tiles grouped by XCD (FATTN_OPT_PF_STAGGER bit 2): traffic and time
run fetch_pf6 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r4f_pfetch6 -o f -- python3 bench.py --prefill-only --pf-stagger 6
run write_pf6 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r4f_pwrite6 -o w -- python3 bench.py --prefill-only --pf-stagger 6
python tools/pmc_summary.py --kernel fattn_pf_kernel --traffic $F/traffic_prefill_xcd.json --bench-line gpurun_out/fetch_pf6.log \
  $(find gpurun_out/r4f_pfetch6 gpurun_out/r4f_pwrite6 -name "*counter_collection.csv") > $F/traffic_prefill_xcd.txt 2>&1
for x in 2 6 2 6; do run pft_$x 120 python bench.py --prefill-only --pf-stagger $x; grep -o '"kernel_ms_avg": [0-9.]*' gpurun_out/pft_$x.log >> $F/prefill_xcd_ab.txt; echo " pf_stagger $x" >> $F/prefill_xcd_ab.txt; done
for f in $(find gpurun_out/r4f_kt -name "*kernel_stats.csv"); do cp "$f" $F/kernel_stats.csv; done
python tools/kstats.py $F/kernel_stats.csv > $F/kernel_stats_summary.txt
ls -la $F; cat $F/kernel_stats_summary.txt $F/traffic_cfg3.txt $F/traffic_prefill.txt $F/traffic_prefill_xcd.txt $F/prefill_xcd_ab.txt $F/bench.json
