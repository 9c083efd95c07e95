#!/usr/bin/env python3
"""Same-box A/B of prefill planner options (diagnostic): bench.py's prefill
measurement (n_q = N = 4096, 32 heads, D = 128; 5 graph-captured launches,
HIP events on the launch stream) for each variant in turn, `--rounds` times.

  python tools/ab_prefill.py --kv q8_0 --mask zero \
      --variant pf8:PF_FORM=1 --variant pf4:PF_FORM=2 --variant inkernel:PF_STAGE=1,PF_FORM=1
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ggml-cuda-experiments_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kv", default="q8_0", choices=["q8_0", "q4_0", "f16"])
    ap.add_argument("--mask", default="zero", choices=["zero", "random", "causal", "none"])
    ap.add_argument("--variant", action="append", default=[], help="name:OPT=val,... (OPT without OPT_)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--H", type=int, default=32)
    args = ap.parse_args()
    import torch
    import fattn
    from bench import hip_events, prefill_measure
    dev = torch.device("cuda", 0)
    hip, evs = hip_events(2)
    variants = []
    for spec in args.variant or ["base:"]:
        name, _, opts = spec.partition(":")
        od = {}
        for kv in filter(None, opts.split(",")):
            k, _, v = kv.partition("=")
            od[getattr(fattn, "OPT_" + k)] = int(v)
        variants.append((name, od))
    res = {n: [] for n, _ in variants}
    for r in range(args.rounds):
        for name, od in variants:
            with fattn.options(od):
                m = prefill_measure(dev, hip, evs, args.kv, args.mask, D=args.D, H=args.H)
            res[name].append(m["kernel_ms_avg"] * 1e3)
            print(f"round {r} {name:12s} {m['kernel_ms_avg'] * 1e3:8.1f} us  frac {m['roofline']['frac']:.4f}  "
                  f"{m['kernel']}", flush=True)
    flops = 4 * (4096 * 4096 if args.mask != "causal" else 4096 * 4097 // 2) * args.D * args.H
    print(f"# prefill kv {args.kv} mask {args.mask} D {args.D} H {args.H}")
    for name, v in res.items():
        med = statistics.median(v)
        print(f"{name:12s} median {med:8.1f} us  min {min(v):8.1f}  max {max(v):8.1f}  "
              f"frac {flops / (med * 1e-6) / 2.5e15:.4f}")


if __name__ == "__main__":
    main()
