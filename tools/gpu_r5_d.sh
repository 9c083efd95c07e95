#!/bin/bash
# Round 5, fourth GPU pass: fattn_pf4_kernel row-level diagnostic over
# diagnostic builds (lib/libfattn_d*.so: plain adds, no scheduling groups, no
# opaque bases, shuffle reductions, all four) to localise its parity failure.
source tools/gpu_round.sh
export TMPDIR=/tmp
for v in dadd dsgb dopq dshf dall; do
  FATTN_LIB=libfattn_$v.so run dbg_$v 120 python -u tools/dbg_pf4.py
done
