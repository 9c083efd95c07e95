#!/bin/bash
# parity + chunk sweep + default stamps (quick iteration)
source tools/gpu_round.sh
export TMPDIR=/tmp
run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
run sweep 600 python tools/sweep_chunk.py
run stamps_c0 200 python tools/stamps.py
run stamps_c512 200 python tools/stamps.py --kv-chunk 512
