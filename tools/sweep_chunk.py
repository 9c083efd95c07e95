"""Time the split kernel for several forced chunk lengths (HIP events around the kernel)."""
import subprocess, sys, json
for ch in [0, 128, 256, 512, 1024, 2048, 4096]:
    out = subprocess.run([sys.executable, "bench.py", "--steps", "100", "--warmup", "10", "--no-cpu-baseline",
                          "--kv-chunk", str(ch)], capture_output=True, text=True)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")]
    if not line:
        print(ch, "FAILED", out.stderr[-500:]); continue
    r = json.loads(line[-1])
    print(f"chunk {ch:5d}: kernel {r['kernel_ms_avg']*1e3:7.2f} us  step {r['ms_per_step']*1e3:7.2f} us  "
          f"achieved {r['roofline']['achieved']:7.1f} GB/s  value {r['value']:7.1f}", flush=True)
