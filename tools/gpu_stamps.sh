#!/bin/bash
# stamp timelines for several split geometries (compute and memory-only builds)
source tools/gpu_round.sh
export TMPDIR=/tmp
for ch in 0 256 512 1024; do
  run stamps_c$ch 200 python tools/stamps.py --kv-chunk $ch
  run nocomp_c$ch 200 python tools/stamps.py --kv-chunk $ch --nocompute
done
