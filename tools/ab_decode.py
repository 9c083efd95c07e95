#!/usr/bin/env python3
"""Same-box A/B of planner options on one decode workload (diagnostic).

Builds the workload once (R rotated KV caches and masks, >= 512 MB per pass,
like bench.py), then for every round times each variant in turn: K launches
captured in one HIP graph, HIP events around the replay on the launch stream,
kernel (+ merge launch) time per step.  Variants alternate, so box drift hits
them alike.  Prints one line per (round, variant) and a median summary.

  python tools/ab_decode.py --workload config3 \
      --variant base: --variant spec:SPLIT_SPEC=2 --variant xcd:SPLIT_XCD=2 --rounds 5
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ggml-cuda-experiments_amd"))
sys.path.insert(0, ROOT)

SHAPES = {
    "config2": dict(kv_type="f16", H=32, Hkv=32, N=2048, NQ=1, D=128),
    "config3": dict(kv_type="q8_0", H=32, Hkv=32, N=4096, NQ=1, D=128),
    "config4": dict(kv_type="q4_0", H=32, Hkv=8, N=8192, NQ=1, D=128),
    "config5": dict(kv_type="q8_0", H=32, Hkv=32, N=4096, NQ=64, D=128),
    "config5_s8": dict(kv_type="q8_0", H=4, Hkv=4, N=4096, NQ=64, D=128),
    "config5_s4": dict(kv_type="q8_0", H=8, Hkv=8, N=4096, NQ=64, D=128),
    "config5_s2": dict(kv_type="q8_0", H=16, Hkv=16, N=4096, NQ=64, D=128),
    "config5_d256": dict(kv_type="q8_0", H=32, Hkv=32, N=4096, NQ=64, D=256),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="config3", choices=sorted(SHAPES))
    ap.add_argument("--variant", action="append", default=[],
                    help="name:OPT=val,OPT=val (OPT without the OPT_ prefix); 'kv_chunk=' sets the chunk")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--lib", default="", help="FATTN_LIB override (a variant library under lib/)")
    for k in ("kv_type", "H", "Hkv", "N", "NQ", "D"):
        ap.add_argument("--" + k, default=None)
    args = ap.parse_args()
    if args.lib:
        os.environ["FATTN_LIB"] = args.lib
    import ctypes as C
    import torch
    import fattn
    from bench import hip_events

    shape = dict(SHAPES[args.workload])
    for k in shape:
        v = getattr(args, k)
        if v is not None:
            shape[k] = v if k == "kv_type" else int(v)
    D, H, Hkv, N, NQ = shape["D"], shape["H"], shape["Hkv"], shape["N"], shape["NQ"]
    typ = fattn.TYPE_NAMES[shape["kv_type"]]
    rb = fattn.row_size(typ, D)
    dev = torch.device("cuda", 0)
    R = max(16, -(-(512 << 20) // (2 * Hkv * N * rb)))
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    kvs = []
    for _ in range(R):
        pair = []
        for _ in range(2):
            x = torch.rand((Hkv * N, D), generator=g, device=dev) * 2 - 1
            pair.append(x.to(torch.float16).view(torch.uint8).reshape(-1) if typ == fattn.TYPE_F16
                        else fattn.quantize(x, typ).reshape(-1))
        kvs.append(pair)
    q = torch.rand((1, NQ, H, D), generator=g, device=dev) * 2 - 1
    npad = (N + 63) // 64 * 64
    masks = [(torch.rand((NQ, npad), generator=g, device=dev) * 2 - 1).to(torch.float16) for _ in range(R)]
    outs = torch.empty((R, 1, NQ, H, D), dtype=torch.float32, device=dev)
    alg = 2 * NQ * H * D * 4 + 2 * Hkv * N * rb + NQ * N * 2

    variants = []
    for spec in args.variant or ["base:"]:
        name, _, opts = spec.partition(":")
        od, chunk = {}, 0
        for kv in filter(None, opts.split(",")):
            k, _, v = kv.partition("=")
            if k == "kv_chunk":
                chunk = int(v)
            else:
                od[getattr(fattn, "OPT_" + k)] = int(v)
        variants.append((name, od, chunk))

    hip, evs = hip_events(2)
    gs = torch.cuda.Stream(dev)
    graphs = []
    for name, od, chunk in variants:
        with fattn.options(od):
            att = fattn.Attention(fattn.q_view(q), fattn.kv_view(kvs[0][0], typ, D, N, Hkv),
                                  fattn.kv_view(kvs[0][1], typ, D, N, Hkv), fattn.mask_view(masks[0]), outs[0],
                                  1.0 / D ** 0.5, kv_chunk=chunk)
            desc = att.describe()

            def step(i):
                att.retarget(k=kvs[i % R][0].data_ptr(), v=kvs[i % R][1].data_ptr(), dst=outs[i % R].data_ptr(),
                             mask=masks[i % R].data_ptr())
                att()

            gs.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(gs):
                for i in range(min(R, 4)):
                    step(i)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=gs):
                for i in range(args.steps):
                    step(i)
        graphs.append((name, gr, desc, att))
        print(f"# {name}: {desc}", flush=True)
    f = C.c_float()
    res = {n: [] for n, *_ in graphs}
    for r in range(args.rounds):
        for name, gr, desc, _ in graphs:
            with torch.cuda.stream(gs):
                gr.replay()
            torch.cuda.synchronize()
            hip.hipEventRecord(evs[0], gs.cuda_stream)
            with torch.cuda.stream(gs):
                gr.replay()
            hip.hipEventRecord(evs[1], gs.cuda_stream)
            torch.cuda.synchronize()
            hip.hipEventElapsedTime(C.byref(f), evs[0], evs[1])
            us = f.value * 1e3 / args.steps
            res[name].append(us)
            print(f"round {r} {name:16s} {us:8.3f} us/step  {alg / us / 1e3:8.1f} GB/s", flush=True)
    print(f"# {args.workload} {shape}  alg bytes {alg}  steps {args.steps}  R {R}")
    for name, v in res.items():
        print(f"{name:16s} median {statistics.median(v):8.3f} us  min {min(v):8.3f}  max {max(v):8.3f}  "
              f"frac {alg / statistics.median(v) / 1e3 / 8000:.4f}")


if __name__ == "__main__":
    main()
