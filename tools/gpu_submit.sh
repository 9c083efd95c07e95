#!/bin/bash
# Submit one GPU command through gpurun; resubmit only while gpurun answers
# "no box / slot free" (exit 3: nothing ran, nothing charged), up to MAX_TRIES (15) times,
# waiting as long as gpurun's back-off message asks (at least 90 s).
# Usage: tools/gpu_submit.sh <log> <timeout_s> <command...>
log=$1; t=$2; shift 2
for i in $(seq 1 ${MAX_TRIES:-15}); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > "$log" 2>&1
  rc=$?
  echo "gpu_submit: try $i rc=$rc" >> "$log"
  [ $rc -ne 3 ] && exit $rc
  w=$(grep -o 'retry in [0-9]*s' "$log" | tail -1 | grep -o '[0-9]*')
  [ -z "$w" ] || [ "$w" -lt 90 ] && w=90
  cp "$log" "$log.try$i"
  sleep $((w + 15))
done
exit 3
