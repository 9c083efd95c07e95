#!/bin/bash
# SQ counters of the multi-query kernel on the prefill shape (separate passes)
source tools/gpu_round.sh
export TMPDIR=/tmp
B="python3 bench.py --n-q 4096 --steps 3 --warmup 1 --rotate 2 --no-cpu-baseline"
run pmc_list 120 rocprofv3 -L
run pmc1 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc1 -o run --output-format csv -- $B
run pmc2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/pmc2 -o run --output-format csv -- $B
run pmc3 300 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT -d gpurun_out/pmc3 -o run --output-format csv -- $B
