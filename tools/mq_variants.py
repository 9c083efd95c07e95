"""Time diagnostic builds of the multi-query kernel (graph replay, no profiler).

  libfattn.so            product
  libfattn_mq_nomem.so   no HBM -> LDS copies (compute + dequant on stale LDS)
  libfattn_mq_nodeq.so   no dequantisation
  libfattn_mq_nocomp.so  copies + dequant + barriers, no MFMA / softmax
Usage: python tools/mq_variants.py
"""
import json
import subprocess
import sys

libs = ["libfattn.so", "libfattn_mq_nomem.so", "libfattn_mq_nodeq.so", "libfattn_mq_nocomp.so", "libfattn_pf_nosm.so"]
import sys as _s
cases = [("prefill", ["--n-q", "4096", "--steps", "5", "--warmup", "1", "--rotate", "2"])]
if "--all" in _s.argv:
    cases = [("c5", ["--n-q", "64", "--steps", "50", "--warmup", "5"]),
             ("c5_1ch", ["--n-q", "64", "--steps", "20", "--warmup", "2", "--kv-chunk", "4096"])] + cases
for name, args in cases:
    for lib in libs:
        env = dict(__import__("os").environ, FATTN_LIB=lib)
        out = subprocess.run([sys.executable, "bench.py", "--no-cpu-baseline"] + args, capture_output=True, text=True,
                             env=env)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(name, lib, "FAILED", out.stderr[-400:], flush=True)
            continue
        r = json.loads(line[-1])
        print(f"{name:8s} {lib:24s} kernel {r['kernel_ms_avg'] * 1e3:9.2f} us  tflops {r['tflops']:8.1f}", flush=True)
