source tools/gpu_round.sh
FATTN_DEBUG=1 run dbgmq 300 python tools/dbg_mq.py
