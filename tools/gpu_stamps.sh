#!/bin/bash
source tools/gpu_round.sh
run stamps_auto 200 python tools/stamps.py
run stamps_256 200 python tools/stamps.py --kv-chunk 256
run stamps_512 200 python tools/stamps.py --kv-chunk 512
run stamps_4096 200 python tools/stamps.py --kv-chunk 4096
