#!/bin/bash
# Round 2's one-off GPU passes, one function per pass (formerly
# tools/gpu_r2_<pass>.sh): bash tools/gpu_r2.sh <pass>
source tools/gpu_round.sh
export TMPDIR=/tmp

# chunk-length sweep for the multi-row configs now that their merge is a second launch
pass_chunks() {
  B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
  rm -f gpurun_out/chunks.txt
  for cfg in "--n-q 64 --heads 4 --kv-heads 4" "--n-q 64" "--kv-type q4_0 --kv-heads 8 --kv-len 8192"; do
    for ch in 0 128 256 512 1024; do
      for w in 0 8; do
        echo "### $cfg --kv-chunk $ch --waves $w" >> gpurun_out/chunks.txt
        timeout -k 10 120 $B $cfg --kv-chunk $ch --waves $w >> gpurun_out/chunks.txt 2>&1 || echo "rc=$?" >> gpurun_out/chunks.txt
      done
    done
  done
  grep -E "###|kernel_ms_avg|rc=" gpurun_out/chunks.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
}

# second-launch merge for multi-row split tiles: parity, then A/B against the fused last-arriver merge
pass_merge() {
  run pytest_m 900 python -u -m pytest tests -m gpu -q --maxfail 20 -p no:cacheprovider --timeout 180 --timeout-method thread
  B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
  rm -f gpurun_out/merge.txt
  for rep in 1; do
    for cfg in "--n-q 64 --heads 4 --kv-heads 4" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "--n-q 64" ""; do
      for v in "" "--fused-merge"; do
        echo "### $cfg $v" >> gpurun_out/merge.txt
        timeout -k 10 120 $B $cfg $v >> gpurun_out/merge.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
      done
    done
  done
  grep -E "###|kernel_ms_avg" gpurun_out/merge.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
}

# planner: two workgroups per CU for long multi-row slices; parity + the decode configs
pass_merge3() {
  run pytest_m 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
  B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
  rm -f gpurun_out/merge3.txt
  for rep in 1 2; do
    for cfg in "--n-q 64" "--n-q 64 --heads 4 --kv-heads 4" "--kv-type q4_0 --kv-heads 8 --kv-len 8192" "" "--kv-type f16 --kv-len 2048"; do
      echo "### $cfg" >> gpurun_out/merge3.txt
      timeout -k 10 120 $B $cfg >> gpurun_out/merge3.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
  done
  grep -E "###|kernel_ms_avg" gpurun_out/merge3.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
}

# multi-query kernel vs split kernel (+ second-launch merge) on batched-decode shapes
pass_mq() {
  run pytest_g 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --maxfail 20 --timeout 180 --timeout-method thread
  B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 200 --rotate 4"
  rm -f gpurun_out/mq.txt
  for cfg in "--n-q 64 --heads 32 --kv-heads 8" "--n-q 128 --heads 32 --kv-heads 8" "--n-q 256" "--n-q 64 --heads 32 --kv-heads 8 --kv-type q4_0" "--n-q 256 --heads 8 --kv-heads 8 --kv-len 8192"; do
    for v in "" "--no-mq"; do
      echo "### $cfg $v" >> gpurun_out/mq.txt
      timeout -k 10 120 $B $cfg $v >> gpurun_out/mq.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
    done
  done
  grep -E "###|kernel_ms_avg" gpurun_out/mq.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
}

# Config-5 per-GPU shard (4 heads, n_q = 64, N = 4096, Q8_0): planner sweep of
# KV chunk x waves x merge form, kernel-only bench lines into gpurun_out/shard/.
pass_shard_sweep() {
  mkdir -p gpurun_out/shard
  B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --workload config5 --heads 4 --kv-heads 4 --steps 200 --warmup 20"
  run planner 120 $B
  grep '^{' gpurun_out/planner.log > gpurun_out/shard/planner.json || true
  for c in 128 256 512 1024; do
    for w in 4 8; do
      for m in "" "--fused-merge"; do
        n=c${c}_w${w}${m:+_fused}
        run $n 120 $B --kv-chunk $c --waves $w $m
        grep '^{' gpurun_out/$n.log > gpurun_out/shard/$n.json || true
      done
    done
  done
  run mq 120 $B --pf 0 --kv-chunk 0
  ls gpurun_out/shard | wc -l
}

# Run-to-run spread on one box: the default bench line three times (config 3),
# then one line per BASELINE.json config 2/4/5 (5 = the 4-head per-GPU shard
# and all 32 heads), kernel-only legs.  Lines land in gpurun_out/spread/.
pass_spread() {
  mkdir -p gpurun_out/spread
  N="--no-cpu-baseline --no-prefill --no-scale-ref"
  for i in 1 2 3; do
    run cfg3_run$i 180 python bench.py $N
    grep '^{' gpurun_out/cfg3_run$i.log > gpurun_out/spread/cfg3_run$i.json || true
  done
  run cfg2 180 python bench.py $N --kv-type f16 --kv-len 2048
  run cfg4 180 python bench.py $N --kv-type q4_0 --kv-heads 8 --kv-len 8192
  run cfg5_shard 180 python bench.py $N --workload config5 --heads 4 --kv-heads 4
  run cfg5_full 180 python bench.py $N --workload config5
  for s in cfg2 cfg4 cfg5_shard cfg5_full; do grep '^{' gpurun_out/$s.log > gpurun_out/spread/$s.json || true; done
  ls -la gpurun_out/spread
}

# one-row tiles: fused workgroup-row merge (default) vs LDS merge + second-launch merge (--wave-merge 1)
pass_wm() {
  B="python bench.py --no-cpu-baseline --no-prefill --no-scale-ref --no-copy-peak --steps 300"
  rm -f gpurun_out/wm.txt
  for rep in 1 2; do
    for cfg in "" "--kv-type f16 --kv-len 2048" "--kv-len 32768 --heads 8 --kv-heads 8" "--waves 4"; do
      for v in "" "--wave-merge 1"; do
        echo "### $cfg $v" >> gpurun_out/wm.txt
        timeout -k 10 120 $B $cfg $v >> gpurun_out/wm.txt 2>&1 || { echo "STOP rc=$?"; exit 1; }
      done
    done
  done
  grep -E "###|kernel_ms_avg" gpurun_out/wm.txt | sed 's/.*"kernel_ms_avg": \([0-9.]*\).*"kernel_ms_median": \([0-9.]*\).*"frac": \([0-9.]*\).*"kernel": "\([^"]*\)".*/  kernel_ms \1 median \2 frac \3 \4/'
}

case "$1" in
  chunks|merge|merge3|mq|shard_sweep|spread|wm) pass_$1 ;;
  *) echo "usage: bash tools/gpu_r2.sh {chunks|merge|merge3|mq|shard_sweep|spread|wm}"; exit 2 ;;
esac
