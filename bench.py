#!/usr/bin/env python3
"""Benchmark the hot path: Q8_0-KV flash-decoding attention on MI355X.

Workload (BASELINE.json metric "attn TFLOPS & HBM GB/s per GPU; head_dim=128
seq=4096 Q8_0 KV", configs[2]): 32 heads, head_dim 128, KV length 4096, one
query row, Q8_0 K and V in ggml block layout (per-head contiguous), f16 mask
row, f32 Q / O.  One step = one FLASH_ATTN_EXT call (split-KV kernel + combine)
over one sequence.  Each step reads a different one of R independent KV caches
(R * 35.7 MB > the 256 MiB Infinity Cache), so the number is HBM, not cache.

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): heads x batch
shard embarrassingly; every rank decodes its own sequence (weak scaling), the
data path has no collective, and after the K timed steps the ranks' outputs are
collected with ONE RCCL all_gather over xGMI (inside the timed region).

Prints ONE JSON line (rank 0).  `value` = whole-job algorithmic bytes / time
(GB/s); `roofline` prices the dominant kernel (fattn_split_kernel) from HIP
events around that kernel alone; `cpu_baseline` times the reference's own CPU
oracle (src/utils.h compiled from /root/reference into oracle/_ref) on a bounded
sample of the same workload; `prefill` (N=1) prices fattn_pf_kernel against
the dense f16 MFMA peak on the compute-bound prefill shape (n_q = N = 4096,
north_star's MFMA-utilisation target), 5 graph-captured launches.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ggml-cuda-experiments_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_F16_PEAK_TFLOPS = 2500.0


def hip_events(n):
    """Raw hipEvent_t handles (torch's Event exposes no handle; the main kernel's
    events are recorded by libfattn on the launch stream)."""
    hip = C.CDLL("libamdhip64.so")
    hip.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    hip.hipEventSynchronize.argtypes = [C.c_void_p]
    hip.hipEventDestroy.argtypes = [C.c_void_p]
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    evs = []
    for _ in range(n):
        e = C.c_void_p()
        assert hip.hipEventCreate(C.byref(e)) == 0
        evs.append(e.value)
    return hip, evs


def cpu_baseline(seconds: float, threads: int):
    """The reference's CPU oracle (kernel_test.h:50-62 calling src/utils.h, built
    from /root/reference into oracle/_ref) on the config-3 shape with the Q8_0
    K/V dequantised to f32 beforehand (dequant not timed).  Repeats the whole
    32-head problem until `seconds` elapse (at least once)."""
    import numpy as np
    from oracle import oracle as orc
    D, H, Hkv, N = 128, 32, 32, 4096
    kind = "reference" if orc.ref_available() else "port"
    orc.srand(1)
    q, k, v, m = (orc.random(n) for n in (D * H, D * N * Hkv, D * N * Hkv, N))
    kq = orc.dequantize(orc.quantize(k.reshape(-1, D), orc.TYPE_Q8_0), orc.TYPE_Q8_0, D).reshape(-1)
    vq = orc.dequantize(orc.quantize(v.reshape(-1, D), orc.TYPE_Q8_0), orc.TYPE_Q8_0, D).reshape(-1)
    reps, t0 = 0, time.perf_counter()
    while True:
        orc.kernel_test_cpu(q, kq, vq, m, N, D, H, Hkv, impl="ref" if kind == "reference" else "oracle",
                            n_threads=threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    bytes_per = (D * H * 4) * 2 + 2 * Hkv * N * (D // 32 * 34) + N * 2
    return {"value": round(bytes_per * reps / el / 1e9, 4), "unit": "GB/s", "cores": threads if kind == "reference" else 1,
            "kind": kind,
            "sample": f"{reps} x full config-3 problem (32 heads x 4096 x 128, Q8_0 K/V dequantised untimed), "
                      f"{el:.1f} s, heads split over {threads} threads, reference src/utils.h loops",
            "ms_per_problem": round(el / reps * 1e3, 2), "host_cpu": _cpu_model()}


def prefill_measure(dev, hip, evs, kvn="q8_0", pf_dequant=0, pf_pipe=0, causal=False, steps=5):
    """The MFMA-bound prefill shape of SURVEY.md §8d (n_q = N = 4096, 32 heads,
    head_dim 128, Q8_0 K/V, random f16 mask, non-causal): `steps` launches of
    fattn_pf_kernel captured in one HIP graph, HIP events around the replay on
    the launch stream.  Two rotated KV caches (compute-bound: the cache state
    barely matters).  Returns the TFLOP/s roofline object."""
    import torch
    import fattn
    D, H, N, NQ, R = 128, 32, 4096, 4096, 2

    typ = fattn.TYPE_NAMES[kvn]
    g = torch.Generator(device=dev)
    g.manual_seed(4321)
    if kvn == "f16":
        kv = [[(torch.rand((H * N, D), generator=g, device=dev) * 2 - 1).to(torch.float16).reshape(-1)
               for _ in range(2)] for _ in range(R)]
    else:
        kv = [[fattn.quantize(torch.rand((H * N, D), generator=g, device=dev) * 2 - 1, typ).reshape(-1)
               for _ in range(2)] for _ in range(R)]
    q = torch.rand((1, NQ, H, D), generator=g, device=dev) * 2 - 1
    mask = (torch.rand((NQ, N), generator=g, device=dev) * 2 - 1).to(torch.float16)
    if causal:  # query i sees keys <= i (N == NQ): the upper triangle is -inf
        tri = torch.triu(torch.ones((NQ, N), dtype=torch.bool, device=dev), diagonal=1)
        mask = mask.masked_fill(tri, float("-inf"))
    out = torch.empty((R, 1, NQ, H, D), dtype=torch.float32, device=dev)
    att = fattn.Attention(fattn.q_view(q), fattn.kv_view(kv[0][0], typ, D, N, H), fattn.kv_view(kv[0][1], typ, D, N, H),
                          fattn.mask_view(mask), out[0], 1.0 / D ** 0.5)

    def step(i):
        att.retarget(k=kv[i % R][0].data_ptr(), v=kv[i % R][1].data_ptr(), dst=out[i % R].data_ptr())
        att()

    gs = torch.cuda.Stream(dev)
    gs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(gs):
        for i in range(2):
            step(i)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=gs):
        for i in range(steps):
            step(i)
    with torch.cuda.stream(gs):
        graph.replay()
    torch.cuda.synchronize()
    f = C.c_float()
    hip.hipEventRecord(evs[0], gs.cuda_stream)
    with torch.cuda.stream(gs):
        graph.replay()
    hip.hipEventRecord(evs[1], gs.cuda_stream)
    torch.cuda.synchronize()
    hip.hipEventElapsedTime(C.byref(f), evs[0], evs[1])
    ms = f.value / steps
    # algorithmic flops: the unmasked (query, key) pairs (all of them without causality)
    pairs = NQ * (NQ + 1) // 2 if causal else NQ * N
    flops = 4 * pairs * D * H
    tf = flops / (ms * 1e-3) / 1e12
    pre = kvn != "f16" and pf_dequant == 2
    f16k = "fattn_pfp_kernel<f16,D128>" if pf_pipe == 2 else "fattn_pf_kernel<f16,D128>"
    kname = (f"pf_dequant_rows_kernel<{kvn}> x2 + {f16k}" if pre
             else f16k if kvn == "f16" else f"fattn_pf_kernel<{kvn},D128>")
    return {"workload": f"prefill_{kvn}_h{H}_d{D}_n{N}_q{NQ}_{'causal' if causal else 'mask'}", "kernel": kname,
            "kernel_ms_avg": round(ms, 5), "flops_per_step": flops,
            "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4), "traffic": None}}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rotate", type=int, default=16, help="independent KV caches cycled through")
    ap.add_argument("--kv-type", default="q8_0", choices=["q8_0", "q4_0", "f16"])
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=0)
    ap.add_argument("--kv-len", type=int, default=4096)
    ap.add_argument("--n-q", type=int, default=1)
    ap.add_argument("--head-dim", type=int, default=128)
    ap.add_argument("--layout", default="head", choices=["head", "pos"])
    ap.add_argument("--kv-chunk", type=int, default=0)
    ap.add_argument("--spw", type=int, default=0, help="split kernel: steps per wave (0 = planner)")
    ap.add_argument("--inflight", type=int, default=0, help="split kernel: steps in flight per wave (0 = planner)")
    ap.add_argument("--no-mask", action="store_true", help="no mask tensor (diagnostics; the metric uses a mask)")
    ap.add_argument("--pf-stagger", type=int, default=2)
    ap.add_argument("--pf-waves", type=int, default=0, help="prefill kernel waves (4 or 8; 0 = library default)")
    ap.add_argument("--pf", type=int, default=0, help="prefill kernel: 0 auto, 1 never, 2 whenever eligible")
    ap.add_argument("--pf-dequant", type=int, default=0,
                    help="quantised prefill: 0 auto, 1 in-kernel dequantisation, 2 f16 pre-pass")
    ap.add_argument("--no-mq", action="store_true", help="never pick the multi-query kernel (split-KV kernel only)")
    ap.add_argument("--split-prio", type=int, default=0,
                    help="split kernel wave priorities: 0 staggered, 1 none, 2 staggered while issuing")
    ap.add_argument("--pf-pipe", type=int, default=0,
                    help="prefill over f16 images: 0 auto, 1 fattn_pf_kernel, 2 software-pipelined fattn_pfp_kernel")
    ap.add_argument("--prefill-causal", action="store_true",
                    help="causal mask on the prefill measurement (fully masked blocks are skipped)")
    ap.add_argument("--prefill-kv", default="q8_0", choices=["q8_0", "q4_0", "f16"],
                    help="K/V type of the prefill measurement (the metric's is q8_0)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prefill", action="store_true", help="skip the prefill-shape MFMA measurement")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import fattn

    if args.spw:
        fattn.set_option(fattn.OPT_SPLIT_STEPS, args.spw)
    if args.inflight:
        fattn.set_option(fattn.OPT_SPLIT_INFLIGHT, args.inflight)
    if args.pf:
        fattn.set_option(fattn.OPT_PF, args.pf)
    fattn.set_option(fattn.OPT_PF_STAGGER, args.pf_stagger)
    if args.pf_waves:
        fattn.set_option(fattn.OPT_PF_WAVES, args.pf_waves)
    if args.pf_dequant:
        fattn.set_option(fattn.OPT_PF_DEQUANT, args.pf_dequant)
    if args.no_mq:
        fattn.set_option(fattn.OPT_MQ_DISABLE, 1)
    if args.split_prio:
        fattn.set_option(fattn.OPT_SPLIT_PRIO, args.split_prio)
    if args.pf_pipe:
        fattn.set_option(fattn.OPT_PF_PIPE, args.pf_pipe)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    D, H, N, NQ = args.head_dim, args.heads, args.kv_len, args.n_q
    Hkv = args.kv_heads or H
    typ = fattn.TYPE_NAMES[args.kv_type]
    rb = fattn.row_size(typ, D)
    R = args.rotate
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)

    # --- synthetic inputs, resident in HBM before timing
    kv_sets = []
    for r in range(R):
        pair = []
        for _ in range(2):
            x = torch.rand((Hkv * N, D), generator=g, device=dev, dtype=torch.float32) * 2 - 1
            if typ == fattn.TYPE_F16:
                pair.append(x.to(torch.float16).view(torch.uint8).reshape(-1))
            else:
                pair.append(fattn.quantize(x, typ).reshape(-1))
            del x
        kv_sets.append(pair)
    q = torch.rand((1, NQ, H, D), generator=g, device=dev) * 2 - 1
    npad = (N + 63) // 64 * 64
    mask = (torch.rand((NQ, npad), generator=g, device=dev) * 2 - 1).to(torch.float16)
    outs = torch.empty((R, 1, NQ, H, D), dtype=torch.float32, device=dev)

    att = fattn.Attention(fattn.q_view(q), fattn.kv_view(kv_sets[0][0], typ, D, N, Hkv, layout=args.layout),
                          fattn.kv_view(kv_sets[0][1], typ, D, N, Hkv, layout=args.layout),
                          None if args.no_mask else fattn.mask_view(mask), outs[0], 1.0 / D ** 0.5,
                          kv_chunk=args.kv_chunk)

    def step(i, stream=None, ev=None):
        kvs = kv_sets[i % R]
        att.retarget(k=kvs[0].data_ptr(), v=kvs[1].data_ptr(), dst=outs[i % R].data_ptr())
        if ev is None:
            att(stream)
        else:
            att(stream, ev[0], ev[1])

    # 1) dominant-kernel duration: eager launches with HIP events recorded by
    #    libfattn around the main kernel only (not part of the timed region)
    n_ev = min(args.steps, 200)
    hip, evs = hip_events(2 * n_ev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for i in range(args.warmup):
        step(i, stream)
    for i in range(n_ev):
        step(i, stream, (evs[2 * i], evs[2 * i + 1]))
    torch.cuda.synchronize()
    f = C.c_float()
    kms = []
    for i in range(n_ev):
        hip.hipEventElapsedTime(C.byref(f), evs[2 * i], evs[2 * i + 1])
        kms.append(f.value)
    kms.sort()
    kern_ms_avg = sum(kms) / len(kms)

    # 2) the timed job: the K steps (step i reads KV cache i % R) captured
    #    back-to-back into one HIP graph -- the launch-bound inner loop lives on
    #    the device, not in Python -- and replayed once inside the timed region.
    #    One step is exactly one launch of fattn_split_kernel (the chunk merge is
    #    fused), so HIP events around the replay on the launch stream give the
    #    kernel's average in-stream duration over the timed region; it agrees
    #    with rocprofv3's per-dispatch average (profiles/).
    K = args.steps
    gs = torch.cuda.Stream(dev)
    gs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(gs):
        for i in range(min(K, R)):
            step(i)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=gs):
        for i in range(K):
            step(i)
    with torch.cuda.stream(gs):
        graph.replay()   # untimed warm replay
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    gathered = torch.empty((world,) + tuple(outs.shape), dtype=torch.float32, device=dev) if world > 1 else None
    ev0, ev1 = evs[0], evs[1]
    t0 = time.perf_counter()
    hip.hipEventRecord(ev0, gs.cuda_stream)
    with torch.cuda.stream(gs):
        graph.replay()   # launches on the current stream: gs, between the events
    hip.hipEventRecord(ev1, gs.cuda_stream)
    if world > 1:
        dist.all_gather_into_tensor(gathered, outs)   # the single RCCL gather over xGMI
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    hip.hipEventSynchronize(ev1)
    kern_ms_eager = kern_ms_avg
    if hip.hipEventElapsedTime(C.byref(f), ev0, ev1) == 0:
        kern_ms_avg = f.value / K          # in-stream average over the timed region
    if world > 1:
        t = torch.tensor([elapsed, kern_ms_avg], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms_avg = float(t[0]), float(t[1])

    bytes_step = (NQ * H * D * 4) * 2 + 2 * Hkv * N * rb + (0 if args.no_mask else NQ * N * 2)
    flops_step = 4 * NQ * N * D * H
    total_bytes = bytes_step * args.steps * world
    value = total_bytes / elapsed / 1e9
    achieved = bytes_step / (kern_ms_avg * 1e-3) / 1e9
    achieved_tf = flops_step / (kern_ms_avg * 1e-3) / 1e12
    # which kernel the planner picks (fattn_api.hip make_plan): the multi-query
    # kernel for quantised K/V with >= 256 packed rows per kv head (16-B layout)
    rk2 = H // Hkv
    heads_ok = NQ * rk2 >= 32 and rk2 <= 64 and rk2 & (rk2 - 1) == 0
    mq_ok = (not args.no_mq and args.kv_type != "f16" and args.layout == "head" and heads_ok and N % 32 == 0)
    pf_ok = mq_ok or (not args.no_mq and args.kv_type == "f16" and args.layout == "head" and heads_ok)
    # the prefill kernel takes it when the 256-row workgroups fill the chip
    pf = (pf_ok and args.pf != 1 and D == 128 and args.kv_chunk <= 0 and N % 64 == 0 and
          (args.pf == 2 or Hkv * ((NQ * rk2 + 255) // 256) >= 256))
    mq = mq_ok and NQ * rk2 >= 256 and not pf
    kname = (f"fattn_pf_kernel<{args.kv_type},D{D}>" if pf else f"fattn_mq_kernel<{args.kv_type},D{D}>" if mq
             else f"fattn_split_kernel<{args.kv_type},{args.kv_type},D{D}>")
    # compute-bound once arithmetic intensity passes the ridge (peak flops / peak bytes)
    mfma_bound = flops_step / bytes_step > MFMA_F16_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9)

    if rank == 0:
        traffic = None
        tf = os.path.join(ROOT, "profiles", "traffic_r01.json")
        if os.path.exists(tf):
            try:
                tj = json.load(open(tf))
                if tj.get("workload") == f"decode_{args.kv_type}_h{H}_hkv{Hkv}_d{D}_n{N}_q{NQ}":
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        res = {
            "metric": "attn TFLOPS & HBM GB/s per GPU; head_dim=128 seq=4096 Q8_0 KV",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f16",
            "data": "synthetic (uniform [-1,1) Q/K/V, K/V quantised on device to ggml blocks; random f16 mask)",
            "config": {"workload": f"decode_{args.kv_type}_h{H}_hkv{Hkv}_d{D}_n{N}_q{NQ}", "heads": H,
                       "kv_heads": Hkv, "head_dim": D, "kv_len": N, "n_q": NQ, "kv_type": args.kv_type,
                       "kv_layout": args.layout, "kv_rotation": R, "parallelism": f"heads_x_batch_shard{world}",
                       "bytes_per_step": bytes_step, "flops_per_step": flops_step},
            "tflops": round(flops_step * args.steps * world / elapsed / 1e12, 4),
            "kernel_ms_avg": round(kern_ms_avg, 5),
            "kernel_ms_eager_avg": round(kern_ms_eager, 5),
            "kernel_timing": "HIP events around the timed graph replay on the launch stream, / steps",
            "roofline": ({"bound": "mfma", "achieved": round(achieved_tf, 2), "peak": MFMA_F16_PEAK_TFLOPS,
                          "unit": "TFLOP/s", "frac": round(achieved_tf / MFMA_F16_PEAK_TFLOPS, 4), "traffic": traffic,
                          "kernel": kname} if mfma_bound else
                         {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kname}),
        }
        if world == 1 and not args.no_prefill and NQ == 1:
            # north_star's second target: MFMA utilisation on the prefill shape
            res["prefill"] = prefill_measure(dev, hip, evs, args.prefill_kv, args.pf_dequant, args.pf_pipe,
                                             args.prefill_causal)
        if world == 1 and not args.no_cpu_baseline and NQ == 1:  # kernel_test.h's CPU path is one query row
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds, min(args.cpu_threads, os.cpu_count() or 1))
        print(json.dumps(res), flush=True)
    for e in evs:
        hip.hipEventDestroy(e)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
