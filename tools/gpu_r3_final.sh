#!/bin/bash
# Round-3 evidence on the final tree: GPU suite, smoke, the default bench line,
# the rocprofv3 kernel-trace summary of the bench, FETCH_SIZE / WRITE_SIZE
# passes (config 3, config 5 on one GPU, its 8-rank shard) turned into
# traffic files tagged with plan + source hash, prefill counter passes, and the
# two-rank rehearsal line.  Summaries land in gpurun_out/final3/.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/final3
mkdir -p $F
[ -n "$PROF_ONLY" ] || run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
[ -n "$PROF_ONLY" ] || run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
if [ -z "$PROF_ONLY" ]; then
  run bench 600 python bench.py
  grep '^{' gpurun_out/bench.log > $F/bench.json || true
  FATTN_BENCH_REHEARSE=1 run rehearse 300 python bench.py --gpus 2 --steps 20 --warmup 5
  grep '^{' gpurun_out/rehearse.log > $F/rehearse_world2.json || true
fi
run kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3_kt -o kt -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
D="--no-cpu-baseline --no-scale-ref --no-copy-peak --no-prefill --steps 50 --warmup 5"
for w in cfg3 cfg5 cfg5shard; do
  X=""; K=fattn_split_kernel
  [ $w = cfg5 ] && X="--workload config5" && K=fattn_bd_kernel
  [ $w = cfg5shard ] && X="--workload config5 --heads 4 --kv-heads 4"
  run fetch_$w 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/prof3_fetch_$w -o f -- python3 bench.py $D $X
  run write_$w 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/prof3_write_$w -o w -- python3 bench.py $D $X
  python tools/pmc_summary.py --kernel $K --traffic $F/traffic_r03_$w.json --bench-line gpurun_out/fetch_$w.log \
    $(find gpurun_out/prof3_fetch_$w gpurun_out/prof3_write_$w -name "*counter_collection.csv") > $F/traffic_$w.txt 2>&1
done
# instruction-mix / wave-state passes for the decode kernels (config 3, config 5, its 8-rank shard)
QA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
QB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
DQ="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5"
for w in cfg3 cfg5 cfg5shard; do
  X=""; K=fattn_split_kernel
  [ $w = cfg5 ] && X="--workload config5" && K=fattn_bd_kernel
  [ $w = cfg5shard ] && X="--workload config5 --heads 4 --kv-heads 4"
  run sqa_$w 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $QA -d gpurun_out/prof3_sqa_$w -o a -- python3 bench.py $DQ $X
  run sqb_$w 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $QB -d gpurun_out/prof3_sqb_$w -o b -- python3 bench.py $DQ $X
  python tools/pmc_summary.py --kernel $K --mfma $(find gpurun_out/prof3_sqa_$w gpurun_out/prof3_sqb_$w -name "*counter_collection.csv") > $F/counters_$w.txt 2>&1
done
P="--no-cpu-baseline --no-scale-ref --no-copy-peak --steps 5 --warmup 2"
run pf_mfma 300 timeout -s KILL 290 rocprofv3 --output-format csv --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/prof3_pfa -o a -- python3 bench.py $P
run pf_wave 300 timeout -s KILL 290 rocprofv3 --output-format csv --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof3_pfb -o b -- python3 bench.py $P
python tools/pmc_summary.py --kernel fattn_pf_kernel --mfma $(find gpurun_out/prof3_pfa gpurun_out/prof3_pfb -name "*counter_collection.csv") > $F/prefill_counters.txt 2>&1
for f in $(find gpurun_out/prof3_kt -name "*kernel_stats.csv"); do cp "$f" $F/kernel_stats.csv; done
python tools/kstats.py $F/kernel_stats.csv > $F/kernel_stats_summary.txt
tail -3 gpurun_out/pytest_gpu.log > $F/pytest_gpu_tail.txt 2>/dev/null
tail -2 gpurun_out/smoke.log > $F/smoke.txt 2>/dev/null
ls -la $F; cat $F/kernel_stats_summary.txt $F/traffic_*.txt $F/prefill_counters.txt $F/counters_*.txt
