#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
run list_counters 120 rocprofv3 -L
run prof_trace 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline
run prof_pmc1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/prof_pmc1 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run prof_pmc2 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT -d gpurun_out/prof_pmc2 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run prof_pmc3 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_pmc3 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run prof_pmc4 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_pmc4 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
