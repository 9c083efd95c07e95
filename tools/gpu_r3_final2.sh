#!/bin/bash
# Round-3 evidence on the final tree (after the granule hand-off and the weak-
# scaling bench): GPU suite, smoke, the default bench line, the two-rank
# rehearsals (batch and head), the rocprofv3 kernel-trace summary of the bench,
# FETCH_SIZE / WRITE_SIZE passes for config 3 (traffic file tagged with plan +
# source hash) and its wave-state counters.  Summaries land in gpurun_out/final4/.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/final4
mkdir -p $F
[ -n "$PROF_ONLY" ] || run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
[ -n "$PROF_ONLY" ] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
if [ -z "$PROF_ONLY" ]; then
  run bench 600 python bench.py
  grep '^{' gpurun_out/bench.log > $F/bench.json || true
  FATTN_BENCH_REHEARSE=1 run rehearse_batch 300 python bench.py --gpus 2 --steps 20 --warmup 5
  grep '^{' gpurun_out/rehearse_batch.log > $F/rehearse_world2_batch.json || true
fi
run kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof4_kt -o kt -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
D="--no-cpu-baseline --no-scale-ref --no-copy-peak --no-prefill --steps 50 --warmup 5"
run fetch_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/prof4_fetch -o f -- python3 bench.py $D
run write_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/prof4_write -o w -- python3 bench.py $D
python tools/pmc_summary.py --kernel fattn_split_kernel --traffic $F/traffic_r03_cfg3.json --bench-line gpurun_out/fetch_cfg3.log \
  $(find gpurun_out/prof4_fetch gpurun_out/prof4_write -name "*counter_collection.csv") > $F/traffic_cfg3.txt 2>&1
QA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
DQ="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5"
run sqa_cfg3 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $QA -d gpurun_out/prof4_sqa -o a -- python3 bench.py $DQ
python tools/pmc_summary.py --kernel fattn_split_kernel --mfma $(find gpurun_out/prof4_sqa -name "*counter_collection.csv") > $F/counters_cfg3.txt 2>&1
for f in $(find gpurun_out/prof4_kt -name "*kernel_stats.csv"); do cp "$f" $F/kernel_stats.csv; done
python tools/kstats.py $F/kernel_stats.csv > $F/kernel_stats_summary.txt
tail -3 gpurun_out/pytest_gpu.log > $F/pytest_gpu_tail.txt 2>/dev/null
tail -2 gpurun_out/smoke.log > $F/smoke.txt 2>/dev/null
ls -la $F; cat $F/kernel_stats_summary.txt $F/traffic_cfg3.txt $F/counters_cfg3.txt $F/bench.json
