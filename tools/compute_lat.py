"""Compute-only latency of the decode step (libfattn_nomem.so: no HBM traffic,
the kernel computes on whatever LDS holds).  Config 3 shape, forced chunk
lengths: chunk = 128*k gives k steps per wave."""
import json, os, subprocess, sys
for lib in ["libfattn_nomem.so", "libfattn_nomem_nopub.so", "libfattn_nomem_notail.so", "libfattn_notail.so"]:
    for ch in [128, 512, 2048, 4096]:
        env = dict(os.environ, FATTN_LIB=lib)
        out = subprocess.run([sys.executable, "bench.py", "--steps", "50", "--warmup", "5", "--no-cpu-baseline",
                              "--kv-chunk", str(ch)] + sys.argv[1:], capture_output=True, text=True, env=env)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if not line:
            print(lib, ch, "FAILED", out.stderr[-300:]); continue
        r = json.loads(line[-1])
        spw = ch // 128
        print(f"{lib} chunk {ch:5d} ({spw} steps/wave): kernel {r['kernel_ms_avg']*1e3:8.2f} us  "
              f"-> {r['kernel_ms_avg']*1e3/spw:6.2f} us per step", flush=True)
