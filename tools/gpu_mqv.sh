source tools/gpu_round.sh
run mqv 600 python tools/mq_variants.py
