"""Time diagnostic builds of the split kernel on config 3 (graph replay, no stamps).

  libfattn.so         product
  libfattn_notail.so  compute, no merge/publish tail
  libfattn_nc.so      memory only (loads + waits), with the tail
  libfattn_nctail.so  memory only, no tail
Usage: python tools/variants.py [--kv-chunk N ...]
"""
import json
import subprocess
import sys

libs = ["libfattn.so", "libfattn_notail.so", "libfattn_nopub.so", "libfattn_noatomic.so", "libfattn_nc.so",
        "libfattn_nctail.so"]
chunks = [int(c) for c in sys.argv[1:]] or [0, 512]
for ch in chunks:
    for lib in libs:
        env = dict(__import__("os").environ, FATTN_LIB=lib)
        out = subprocess.run([sys.executable, "bench.py", "--steps", "100", "--warmup", "10", "--no-cpu-baseline",
                              "--kv-chunk", str(ch)], capture_output=True, text=True, env=env)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(ch, lib, "FAILED", out.stderr[-400:])
            continue
        r = json.loads(line[-1])
        print(f"chunk {ch:5d} {lib:20s} step {r['ms_per_step'] * 1e3:7.2f} us  kernel(event) {r['kernel_ms_avg'] * 1e3:7.2f} us",
              flush=True)
