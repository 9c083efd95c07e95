#!/bin/bash
source tools/gpu_round.sh
run prims 300 python -m pytest tests/test_gpu_prims.py -q -s -p no:cacheprovider
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
