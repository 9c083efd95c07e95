#!/bin/bash
# Round 3: the whole GPU suite (one process), then the bd masked probe.
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread
run dbg_bd 240 python -u tools/dbg_bd.py
