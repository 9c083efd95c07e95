#!/bin/bash
# Round 3: bd kernel A/B (product vs raw-1-late prologue) on config 5 full and
# shard, after the bd parity subset.
source tools/gpu_round.sh
export TMPDIR=/tmp
D=${OUT:-r3bd5}
mkdir -p gpurun_out/$D
run pytest_bd 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bd or config5"
N="--no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 100 --warmup 10"
for rep in 1 2; do
for lib in libfattn.so; do
  for c in full shard; do
    X=""; [ $c = shard ] && X="--heads 4 --kv-heads 4"
    n=${lib%.so}_${c}_$rep
    FATTN_LIB=$lib run kt_$n 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$D/$n -o k -- python3 bench.py $N --workload config5 $X
  done
done
done
python tools/kstats.py $(find gpurun_out/$D -name "*kernel_stats.csv" | sort) > gpurun_out/$D/summary.txt
run st_full 120 python tools/stamps_bd.py --heads 32
cp gpurun_out/st_full.log gpurun_out/$D/
cat gpurun_out/$D/summary.txt
