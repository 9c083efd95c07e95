#!/bin/bash
# Round 5: kernel stats of the staged prefill (stage + flags + f16 body), then
# the instruction-mix / LDS counters of the prefill body and of the role-form
# batched decode (config 5, new image swizzles) -- the round-4 counter sets.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r5g
mkdir -p $F
run pfstats 200 timeout -s KILL 190 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5g_prof/pf -o pf -- python3 bench.py --prefill-only
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run pfA 200 timeout -s KILL 190 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r5g_pmc/pfA -o a -- python3 bench.py --prefill-only
run pfB 200 timeout -s KILL 190 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r5g_pmc/pfB -o b -- python3 bench.py --prefill-only
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5 --workload config5"
run c5A 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r5g_pmc/c5A -o a -- python3 bench.py $B
run c5B 150 timeout -s KILL 140 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r5g_pmc/c5B -o b -- python3 bench.py $B
python tools/pmc_summary.py --kernel fattn_pf_kernel --mfma $(find gpurun_out/r5g_pmc/pfA gpurun_out/r5g_pmc/pfB -name "*counter_collection.csv") > $F/counters_prefill.txt 2>&1
python tools/pmc_summary.py --kernel fattn_bdp_kernel --mfma $(find gpurun_out/r5g_pmc/c5A gpurun_out/r5g_pmc/c5B -name "*counter_collection.csv") > $F/counters_cfg5_bdp.txt 2>&1
python tools/kstats.py $(find gpurun_out/r5g_prof/pf -name "*kernel_stats.csv") > $F/prefill_kernel_stats.txt 2>&1 || true
cat $F/counters_prefill.txt $F/counters_cfg5_bdp.txt $F/prefill_kernel_stats.txt
# per-phase cycles of the 8-wave f16 body (stamps build), no mask
run pf_stamps_f16 200 python -u tools/pf_stamps.py --no-mask --kv-type f16
