#!/bin/bash
# Submit one GPU command through gpurun; resubmit only while gpurun answers
# "no box / slot free" (exit 3: nothing ran, nothing charged), up to 15 times.
# Usage: tools/gpu_submit.sh <log> <timeout_s> <command...>
log=$1; t=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  echo "gpu_submit: try $i rc=$rc" >> "$log"
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
