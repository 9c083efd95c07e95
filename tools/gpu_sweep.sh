#!/bin/bash
source tools/gpu_round.sh
export TMPDIR=/tmp
run sweep 600 python tools/sweep_chunk.py
run prof_pmc1 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/prof_pmc1 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
