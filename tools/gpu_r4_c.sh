#!/bin/bash
# Round 4: where config 5's batched-decode time goes, both forms (--bd 2 the
# all-waves kernel, --bd 3 the compute / build-role kernel): per-wave phase
# stamps (diagnostic library libfattn_stamps.so) and counter passes.
source tools/gpu_round.sh
export TMPDIR=/tmp
F=gpurun_out/r4c
mkdir -p $F
run st_bdp 200 python tools/stamps_bd.py --form bdp --heads 32
run st_bd 200 python tools/stamps_bd.py --form bd --heads 32
cp gpurun_out/st_bdp.log $F/stamps_cfg5_bdp.txt; cp gpurun_out/st_bd.log $F/stamps_cfg5_bd.txt
B="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 20 --warmup 5 --workload config5"
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for f in 3 2; do
  run pmcA_$f 120 timeout -s KILL 100 rocprofv3 --output-format csv --pmc $A -d gpurun_out/r4c_pmc/A_$f -o a -- python3 bench.py $B --bd $f
  run pmcB_$f 120 timeout -s KILL 100 rocprofv3 --output-format csv --pmc $P -d gpurun_out/r4c_pmc/B_$f -o b -- python3 bench.py $B --bd $f
done
run fetch_3 120 timeout -s KILL 100 rocprofv3 --output-format csv --pmc FETCH_SIZE -d gpurun_out/r4c_pmc/F_3 -o f -- python3 bench.py $B --bd 3
run write_3 120 timeout -s KILL 100 rocprofv3 --output-format csv --pmc WRITE_SIZE -d gpurun_out/r4c_pmc/W_3 -o w -- python3 bench.py $B --bd 3
python tools/pmc_summary.py --kernel fattn_bdp_kernel --mfma $(find gpurun_out/r4c_pmc/A_3 gpurun_out/r4c_pmc/B_3 -name "*counter_collection.csv") > $F/counters_cfg5_bdp.txt 2>&1
python tools/pmc_summary.py --kernel fattn_bd_kernel --mfma $(find gpurun_out/r4c_pmc/A_2 gpurun_out/r4c_pmc/B_2 -name "*counter_collection.csv") > $F/counters_cfg5_bd.txt 2>&1
python tools/pmc_summary.py --kernel fattn_bdp_kernel --traffic $F/traffic_cfg5_bdp.json --bench-line gpurun_out/fetch_3.log \
  $(find gpurun_out/r4c_pmc/F_3 gpurun_out/r4c_pmc/W_3 -name "*counter_collection.csv") > $F/traffic_cfg5_bdp.txt 2>&1
cat $F/stamps_cfg5_bdp.txt $F/stamps_cfg5_bd.txt $F/counters_cfg5_bdp.txt $F/counters_cfg5_bd.txt $F/traffic_cfg5_bdp.txt
