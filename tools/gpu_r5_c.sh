#!/bin/bash
# Round 5, third GPU pass: fattn_pf4_kernel row-level diagnostic, then the
# default bench line of the current tree.
source tools/gpu_round.sh
export TMPDIR=/tmp
run dbg_pf4 200 python -u tools/dbg_pf4.py
run bench 500 python -u bench.py
