#!/bin/bash
source tools/gpu_round.sh
run dbg_q4 200 python tools/dbg_q4.py
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider -k "not test_quantize_bitexact"
