"""Time the decode kernel for several forced chunk lengths (graph replay + HIP events).
Usage: python tools/sweep_chunk.py [bench.py workload args...]"""
import json
import subprocess
import sys

extra = sys.argv[1:]
for ch in [0, 128, 256, 512, 1024, 2048]:
    out = subprocess.run([sys.executable, "bench.py", "--steps", "100", "--warmup", "10", "--no-cpu-baseline",
                          "--kv-chunk", str(ch)] + extra, capture_output=True, text=True)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(ch, "FAILED", out.stderr[-500:]); continue
    r = json.loads(line[-1])
    print(f"{' '.join(extra) or 'config3'} chunk {ch:5d}: kernel {r['kernel_ms_avg']*1e3:7.2f} us  step {r['ms_per_step']*1e3:7.2f} us  "
          f"achieved {r['roofline']['achieved']:7.1f} GB/s  value {r['value']:7.1f}", flush=True)
