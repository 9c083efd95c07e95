#!/bin/bash
# Round-6 evidence on the final tree (two calls): PART=tests -- the GPU suite
# and smoke; PART=prof -- the default bench line, the rocprofv3 kernel-trace
# summary of the bench, the FETCH_SIZE / WRITE_SIZE passes (traffic files
# tagged with plan + source hash) for config 3 and for the prefill shape (the
# pre-pass and the body summed per launch), and the instruction-mix counters of the
# prefill body and of the config-5 role-form kernel.  Summaries land in
# gpurun_out/r6final/.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r6final
mkdir -p $F
if [ "$PART" = tests ]; then
  run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
  run smoke 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  tail -3 gpurun_out/pytest_gpu.log > $F/pytest_gpu_tail.txt 2>/dev/null
  tail -2 gpurun_out/smoke.log > $F/smoke.txt 2>/dev/null
  cat $F/pytest_gpu_tail.txt $F/smoke.txt
  exit 0
fi
run bench 600 python bench.py
grep '^{' gpurun_out/bench.log > $F/bench.json || true
run kt 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6f_kt -o kt -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
python tools/kstats.py $(find gpurun_out/r6f_kt -name "*kernel_stats.csv") $(find gpurun_out/r6f_kt -name "*kernel_trace.csv") > $F/kernel_stats_summary.txt 2>&1 || true
D="--no-cpu-baseline --no-scale-ref --no-copy-peak --no-prefill --steps 50 --warmup 5"
run fetch_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r6f_fetch -o f -- python3 bench.py $D
run write_cfg3 180 timeout -s KILL 170 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r6f_write -o w -- python3 bench.py $D
python tools/pmc_summary.py --kernel fattn_split_kernel --traffic $F/traffic_r06_cfg3.json --bench-line gpurun_out/fetch_cfg3.log \
  $(find gpurun_out/r6f_fetch gpurun_out/r6f_write -name "*counter_collection.csv") > $F/traffic_cfg3.txt 2>&1
run fetch_pf 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r6f_pfetch -o f -- python3 bench.py --prefill-only
run write_pf 240 timeout -s KILL 230 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r6f_pwrite -o w -- python3 bench.py --prefill-only
python tools/pmc_summary.py --kernel pf_prepass_kernel,fattn_pf4_kernel --sum-kernels \
  --traffic $F/traffic_r06_prefill.json --bench-line gpurun_out/fetch_pf.log \
  $(find gpurun_out/r6f_pfetch gpurun_out/r6f_pwrite -name "*counter_collection.csv") > $F/traffic_prefill.txt 2>&1
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run pfA 200 timeout -s KILL 190 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r6f_pmc/pfA -o a -- python3 bench.py --prefill-only
run pfB 200 timeout -s KILL 190 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r6f_pmc/pfB -o b -- python3 bench.py --prefill-only
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5 --workload config5"
run c5A 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r6f_pmc/c5A -o a -- python3 bench.py $B
run c5B 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r6f_pmc/c5B -o b -- python3 bench.py $B
python tools/pmc_summary.py --kernel fattn_pf4_kernel --mfma $(find gpurun_out/r6f_pmc/pfA gpurun_out/r6f_pmc/pfB -name "*counter_collection.csv") > $F/counters_prefill.txt 2>&1
python tools/pmc_summary.py --kernel fattn_bdp_kernel --mfma $(find gpurun_out/r6f_pmc/c5A gpurun_out/r6f_pmc/c5B -name "*counter_collection.csv") > $F/counters_cfg5_bdp.txt 2>&1
cat $F/kernel_stats_summary.txt $F/traffic_cfg3.txt $F/traffic_prefill.txt $F/counters_prefill.txt $F/counters_cfg5_bdp.txt
