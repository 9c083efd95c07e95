#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per counter set; at most 8 SQ and 2
# GRBM counters each) on config 3 (split kernel) and config 5 (batched-decode
# kernel, all 32 heads): wave-cycle breakdown, instruction mix, LDS conflicts.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3pmc}
mkdir -p gpurun_out/$D
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for w in cfg3 cfg5; do
  X=""; [ $w = cfg5 ] && X="--workload config5"
  run pmcA_$w 120 timeout -s KILL 100 rocprofv3 --output-format csv --pmc $A -d gpurun_out/$D/A_$w -o a -- python3 bench.py $B $X
  run pmcB_$w 120 timeout -s KILL 100 rocprofv3 --output-format csv --pmc $P -d gpurun_out/$D/B_$w -o b -- python3 bench.py $B $X
done
for w in cfg3 cfg5; do
  K=fattn_split_kernel; [ $w = cfg5 ] && K=fattn_bd_kernel
  python tools/pmc_summary.py --kernel $K --mfma $(find gpurun_out/$D -path "*_$w*" -name "*counter_collection.csv") > gpurun_out/$D/summary_$w.txt 2>&1
  cat gpurun_out/$D/summary_$w.txt
done
