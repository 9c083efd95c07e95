#!/usr/bin/env python3
"""Benchmark the hot path: Q8_0-KV flash-decoding attention on MI355X.

One GPU (default; BASELINE.json metric "attn TFLOPS & HBM GB/s per GPU;
head_dim=128 seq=4096 Q8_0 KV", configs[2]): 32 heads, head_dim 128, KV length
4096, one query row, Q8_0 K and V in ggml block layout (per-head contiguous),
f16 mask row, f32 Q / O.  One step = one FLASH_ATTN_EXT call (one launch: the
split-KV chunk merge is fused) over the whole problem.  Each step reads a
different one of R independent KV caches (R * 35.7 MB > the 256 MiB Infinity
Cache), so the number is HBM, not cache.

N GPUs (`--gpus N`, or launched by torch.distributed.run): heads x batch
sharding.  The value line is BASELINE.json configs[4] --
n_q = 64 query rows, 32 heads, N = 4096, Q8_0 -- as ONE problem head-sharded
over the ranks (strong scaling; rank r owns kv heads [r*Hkv/N, (r+1)*Hkv/N)
and their q heads, zero-copy slices, fattn.shard): every timed step is the
rank's FLASH_ATTN_EXT followed by the RCCL all_gather over xGMI of that step's
output and its permute into the ggml dst layout, K gathers inside the timed
region.  value = the config-5 bytes x K / the slowest rank's wall time.  The
N = 1 line carries `strong_scaling_ref` (config 5 on one GPU) as the
denominator.  Beside the value line: `kernel_only` (the same launches with no
gather, graph-replayed: SURVEY's "near-linear applies to the kernel part") and
`weak_scaling_config3` (every rank decodes its own config-3 sequence, one
gather per step; `--multi batch` makes that the value line).  `--gpus N` with
no launcher starts N child ranks itself (before touching the GPU).

Prints ONE JSON line (rank 0).  `value` = whole-job algorithmic bytes / wall
time (GB/s); `roofline` prices the dominant kernel from HIP events on its
launch stream; `cpu_baseline` times the reference's own CPU oracle
(src/utils.h compiled from /root/reference into oracle/_ref) on the host
cores, single-thread and on the box's thread share, median of >= 5 runs;
`prefill` (N=1) prices fattn_pf_kernel against the dense f16 MFMA peak on the
compute-bound prefill shape (n_q = N = 4096, north_star's MFMA target).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ggml-cuda-experiments_amd"))
sys.path.insert(0, ROOT)

ROTATE_BYTES = 512 << 20  # KV bytes one rank reads per pass of the rotation
HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
MFMA_F16_PEAK_TFLOPS = 2500.0
METRIC = "attn TFLOPS & HBM GB/s per GPU; head_dim=128 seq=4096 Q8_0 KV"

# BASELINE.json configs used as bench workloads (the others are parity cases)
WORKLOADS = {
    "config3": dict(kv_type="q8_0", heads=32, kv_heads=32, kv_len=4096, n_q=1, head_dim=128),
    "config5": dict(kv_type="q8_0", heads=32, kv_heads=32, kv_len=4096, n_q=64, head_dim=128),
}


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


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float, threads: int):
    """The reference's CPU oracle (kernel_test.h:50-62 calling src/utils.h:5-49,
    built from /root/reference into oracle/_ref; the restated oracle when that
    library is absent) on the config-3 shape, Q8_0 K/V dequantised to f32
    beforehand (not timed).  Two modes: (i) one thread, exactly the
    reference's loops; (ii) heads split over `threads` threads.  Each mode:
    the whole 32-head problem repeated >= 5 times within ~seconds/2; median."""
    from oracle import oracle as orc
    D, H, Hkv, N = 128, 32, 32, 4096
    kind = "reference" if orc.ref_available() else "port"
    orc.srand(1)
    q, k, v, m = (orc.random(n) for n in (D * H, D * N * Hkv, D * N * Hkv, N))
    kq = orc.dequantize(orc.quantize(k.reshape(-1, D), orc.TYPE_Q8_0), orc.TYPE_Q8_0, D).reshape(-1)
    vq = orc.dequantize(orc.quantize(v.reshape(-1, D), orc.TYPE_Q8_0), orc.TYPE_Q8_0, D).reshape(-1)
    bytes_per = (D * H * 4) * 2 + 2 * Hkv * N * (D // 32 * 34) + N * 2

    def mode(nt):
        runs, t_all = [], time.perf_counter()
        while len(runs) < 5 or (time.perf_counter() - t_all < seconds / 2 and len(runs) < 200):
            t0 = time.perf_counter()
            orc.kernel_test_cpu(q, kq, vq, m, N, D, H, Hkv, impl="ref" if kind == "reference" else "oracle",
                                n_threads=nt)
            runs.append(time.perf_counter() - t0)
        med = statistics.median(runs)
        return {"value": round(bytes_per / med / 1e9, 4), "unit": "GB/s", "cores": nt, "runs": len(runs),
                "ms_per_problem_median": round(med * 1e3, 2)}

    single = mode(1)
    multi = mode(threads)
    return {**multi, "kind": kind,
            "sample": f"full config-3 problem (32 heads x 4096 x 128, Q8_0 K/V dequantised untimed), median of "
                      f"{multi['runs']} runs, heads split over {threads} threads (the box's thread share: "
                      f"OMP_NUM_THREADS; nproc reports the whole host), reference src/utils.h loops",
            "single_thread": single, "nproc": os.cpu_count(), "host_cpu": _cpu_model()}


def measured_hbm_peaks():
    """Measured HBM ceilings for the roofline's secondary fractions (BASELINE.md:
    fraction against a measured copy-kernel peak): tools/hbm_copy.hip built into
    lib/libhbmcopy.so -- a global_load_dwordx4 / global_store_dwordx4 copy of
    1 GiB (read + written bytes / median launch time, the form of
    MI355X_MICROARCH.md's 6.29 TB/s float4-copy figure) and a dwordx4 read-only
    stream of the same buffer (the decode kernel's access mix is read-only)."""
    path = os.path.join(ROOT, "ggml-cuda-experiments_amd", "lib", "libhbmcopy.so")
    if not os.path.exists(path):
        return None
    import torch  # noqa: F401  (the probe binds to torch's HIP runtime)
    L = C.CDLL(path)
    L.hbm_probe.restype = C.c_int
    L.hbm_probe.argtypes = [C.c_size_t, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    cp, rd = C.c_float(), C.c_float()
    if L.hbm_probe(1 << 30, 10, C.byref(cp), C.byref(rd)) != 0:
        return None
    return {"copy_dwordx4": round(cp.value, 1), "read_dwordx4": round(rd.value, 1)}


def oneshot_ceiling(shape):
    """The one-shot read ceiling of THIS launch shape (tools/hbm_copy.hip
    hbm_oneshot): the same 256 workgroups each reading its contiguous slice of
    the K cache and of the V cache once -- nothing else in the launch -- over 16
    rotated cache pairs, back-to-back launches, HIP events.  Two load forms (all
    of a workgroup's share in flight): LDS-DMA from 8 waves, and
    global_load_dwordx4 into registers from 8 and 16 waves; the fastest is the
    ceiling.  Config-3-shaped workloads only (Hkv x 8 chunks = 256 workgroups
    of whole KiB), else None."""
    import fattn
    path = os.path.join(ROOT, "ggml-cuda-experiments_amd", "lib", "libhbmcopy.so")
    typ = fattn.TYPE_NAMES[shape["kv_type"]]
    per = shape["kv_len"] * fattn.row_size(typ, shape["head_dim"]) // 8
    if not os.path.exists(path) or shape["kv_heads"] * 8 != 256 or per % 1024 or per // 1024 > 160:
        return None
    L = C.CDLL(path)
    if not hasattr(L, "hbm_oneshot"):
        return None
    L.hbm_oneshot.restype = C.c_float
    L.hbm_oneshot.argtypes = [C.c_uint, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    forms = {"ldsdma_8waves": (8, 0), "vgpr_8waves": (8, 2), "vgpr_16waves": (16, 2)}
    us = {}
    for name, (w, mode) in forms.items():
        t = [L.hbm_oneshot(per, 256, w, mode, 16, 200) for _ in range(3)]
        t = [x for x in t if x > 0]
        if t:
            us[name] = round(min(t), 3)
    if not us:
        return None
    best = min(us, key=us.get)
    return {"us_per_launch": us, "best": best, "kv_bytes": 2 * 256 * per}


def source_hash():
    """Hash of the kernel sources + ABI header: tags the committed PMC traffic so
    a changed kernel never reports stale bytes."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "ggml-cuda-experiments_amd", "csrc")
    for f in sorted(os.listdir(csrc)) + ["../../include/fattn.h", "../../include/fattn_debug.h"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()[:16]


def committed_traffic(workload, kernel):
    """PMC traffic (profiles/traffic_*.json, tools/pmc_summary.py --traffic) for
    this workload, only if it was measured on this exact kernel plan (describe
    string) and kernel sources (source_hash); else None."""
    import glob
    for tf in sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_*.json")), reverse=True):
        try:
            tj = json.load(open(tf))
        except (OSError, ValueError):
            continue
        if (tj.get("workload") == workload and tj.get("plan") == kernel and
                tj.get("source_hash") == source_hash()):
            return tj.get("hbm_bytes_per_launch")
    return None


def cpu_baseline_prefill(rows=256):
    """Prefill-shape CPU baseline (one head timed, extrapolation
    labelled): the reference's own mulmat_cpu / softmax (src/utils.h:5-49,
    oracle/_ref; the restated oracle when that library is absent) for ONE head
    of the prefill shape (N = 4096 keys, D = 128) over `rows` of its 4096 query
    rows, single thread; scaled linearly to 4096 rows x 32 heads."""
    from oracle import oracle as orc
    D, N, NQ, H = 128, 4096, 4096, 32
    impl = "ref" if orc.ref_available() else "oracle"
    rng = np.random.default_rng(7)
    q = (1 - 2 * rng.random((rows, D), dtype=np.float32)).astype(np.float32)
    k = (1 - 2 * rng.random((N, D), dtype=np.float32)).astype(np.float32)
    v = (1 - 2 * rng.random((N, D), dtype=np.float32)).astype(np.float32)
    m = (1 - 2 * rng.random(N, dtype=np.float32)).astype(np.float32)
    t0 = time.perf_counter()
    s = orc.mulmat_f32(q, k, m, rows, N, D, 1.0 / np.sqrt(np.float32(D)), True, impl=impl)
    p = orc.softmax(s, N, rows, impl=impl)
    orc.mulmat_f32(p, v, None, rows, D, N, 1.0, False, impl=impl)
    dt = time.perf_counter() - t0
    flops = 4 * rows * N * D
    full_s = dt * (NQ / rows) * H
    return {"value": round(flops / dt / 1e9, 4), "unit": "GFLOP/s", "cores": 1,
            "kind": "reference" if impl == "ref" else "port",
            "sample": f"1 head x {rows} of 4096 query rows x 4096 keys x D 128 (src/utils.h mulmat_cpu (Q.K^T, "
                      f"B transposed) + softmax + mulmat_cpu (P.V)), one thread, {dt:.2f} s; the mask row is "
                      f"broadcast over rows as mulmat_cpu's f32 form does",
            "extrapolated_full_prefill_s": round(full_s, 1),
            "extrapolation": f"linear: x {NQ // rows} rows x {H} heads (not measured)"}


def seq64_measure(dev, hip, evs, steps=20, S=64, H=32, N=4096, D=128, kvn="q8_0"):
    """SURVEY.md §8d's alternative reading of config 5, reported as a labelled
    extra: 64 independent sequences (ggml ne03 = 64), one query row each, each
    with its own 4096-position Q8_0 cache -- 2.28 GB of K + V per step, read
    once (a step alone is 9x the 256 MiB Infinity Cache: no rotation needed).
    The mask row is broadcast over the sequences (ggml's ne32 = 1).  `steps`
    launches captured in one HIP graph, HIP events around the replay on the
    launch stream."""
    import torch
    import fattn
    typ = fattn.TYPE_NAMES[kvn]
    rb = fattn.row_size(typ, D)
    g = torch.Generator(device=dev)
    g.manual_seed(6464)
    kv = []
    for _ in range(2):  # K, V: [S][H][N][row], quantised one sequence at a time
        buf = torch.empty((S, H * N * rb), dtype=torch.uint8, device=dev)
        for s_ in range(S):
            x = torch.rand((H * N, D), generator=g, device=dev, dtype=torch.float32) * 2 - 1
            buf[s_].copy_(fattn.quantize(x, typ).reshape(-1))
            del x
        kv.append(buf.reshape(-1))
    q = torch.rand((S, 1, H, D), generator=g, device=dev) * 2 - 1
    mask = (torch.rand((1, (N + 63) // 64 * 64), generator=g, device=dev) * 2 - 1).to(torch.float16)
    out = torch.empty((S, 1, H, D), dtype=torch.float32, device=dev)
    att = fattn.Attention(fattn.q_view(q), fattn.kv_view(kv[0], typ, D, N, H, S), fattn.kv_view(kv[1], typ, D, N, H, S),
                          fattn.mask_view(mask), out, 1.0 / D ** 0.5)
    gs = torch.cuda.Stream(dev)
    gs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(gs):
        for _ in range(2):
            att()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=gs):
        for _ in range(steps):
            att()
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
    alg = 2 * S * H * N * rb + 2 * S * H * D * 4 + N * 2  # K + V + Q + O + the broadcast mask row
    gbs = alg / (ms * 1e-3) / 1e9
    res = {"workload": f"decode_{kvn}_h{H}_d{D}_n{N}_q1_s{S}", "kernel": att.describe(), "kernel_ms_avg": round(ms, 5),
           "bytes_per_step": alg, "value": round(gbs, 2), "unit": "GB/s",
           "roofline": {"bound": "hbm", "achieved": round(gbs, 2), "peak": 8000.0, "unit": "GB/s",
                        "frac": round(gbs / 8000.0, 4)},
           "note": "SURVEY.md 8(d)'s alternative reading of config 5, labelled as an extra: 64 independent "
                   "sequences (ne03 = 64), one query row each, each its own 4096-position Q8_0 cache"}
    del kv, q, out, att, graph
    torch.cuda.empty_cache()
    return res


def prefill_measure(dev, hip, evs, kvn="q8_0", mask_kind="zero", steps=5, D=128, H=32, reps=3):
    """The MFMA-bound prefill shape of SURVEY.md §8d (n_q = N = 4096, 32 heads,
    head_dim 128, Q8_0 K/V, non-causal, an f16 mask of zeros -- "zero mask":
    every key visible; "random": U[-1,1) like kernel_test.h:48; "causal": 0 on
    and below the diagonal, -inf above): `steps` launches captured in one HIP
    graph, HIP events around each of `reps` replays on the launch stream, the
    median replay reported (all of them in kernel_ms_reps).  Two rotated KV
    caches (compute-bound: the cache state barely matters).  The pre-pass
    (pf_prepass_kernel: K / V staged to f16, live / all-zero mask block flags)
    is inside the timed region.  (D / H: other head dims for tools/ab_prefill.py; the bench line
    is D = 128, H = 32.)"""
    import torch
    import fattn
    N, NQ, R = 4096, 4096, 2

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
    causal = mask_kind == "causal"
    if mask_kind == "random":
        mask = (torch.rand((NQ, N), generator=g, device=dev) * 2 - 1).to(torch.float16)
    else:
        mask = torch.zeros((NQ, N), dtype=torch.float16, device=dev)
    if causal:  # query i sees keys <= i (N == NQ): the upper triangle is -inf
        tri = torch.triu(torch.ones((NQ, N), dtype=torch.bool, device=dev), diagonal=1)
        mask = mask.masked_fill(tri, float("-inf"))
    out = torch.empty((R, 1, NQ, H, D), dtype=torch.float32, device=dev)
    att = fattn.Attention(fattn.q_view(q), fattn.kv_view(kv[0][0], typ, D, N, H), fattn.kv_view(kv[0][1], typ, D, N, H),
                          None if mask_kind == "none" else fattn.mask_view(mask), out[0], 1.0 / D ** 0.5)

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
    # `reps` timed replays, the median reported (one replay of 5 launches moved
    # by +-5 % from replay to replay on one box: DVFS)
    f = C.c_float()
    reps_ms = []
    for _ in range(reps):
        hip.hipEventRecord(evs[0], gs.cuda_stream)
        with torch.cuda.stream(gs):
            graph.replay()
        hip.hipEventRecord(evs[1], gs.cuda_stream)
        torch.cuda.synchronize()
        hip.hipEventElapsedTime(C.byref(f), evs[0], evs[1])
        reps_ms.append(f.value / steps)
    ms = sorted(reps_ms)[len(reps_ms) // 2]
    # algorithmic flops: the unmasked (query, key) pairs (all of them without causality)
    pairs = NQ * (NQ + 1) // 2 if causal else NQ * N
    flops = 4 * pairs * D * H
    tf = flops / (ms * 1e-3) / 1e12
    # algorithmic bytes: Q + K + V + mask + O at stored precision, once each
    alg_bytes = 2 * NQ * H * D * 4 + 2 * H * N * fattn.row_size(typ, D) + (0 if mask_kind == "none" else NQ * N * 2)
    workload = f"prefill_{kvn}_h{H}_d{D}_n{N}_q{NQ}_{mask_kind}_mask"
    kname = att.describe()
    # HBM bytes per launch from the committed FETCH_SIZE / WRITE_SIZE passes of
    # this exact plan and source (tools/pmc_summary.py --traffic), else None
    traffic = committed_traffic(workload, kname)
    return {"workload": workload, "kernel": kname, "kernel_ms_avg": round(ms, 5),
            "kernel_ms_reps": [round(x, 5) for x in reps_ms], "flops_per_step": flops,
            "bytes_per_step": alg_bytes,
            "roofline": {"bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / MFMA_F16_PEAK_TFLOPS, 4), "traffic": traffic,
                         "traffic_over_algorithmic": round(traffic / alg_bytes, 4) if traffic else None}}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="auto", choices=["auto", "config3", "config5"],
                    help="auto: config3 (on every rank with --multi batch), config5 with --multi head")
    ap.add_argument("--multi", default="head", choices=["batch", "head"],
                    help="N > 1: head = BASELINE config 5 as one problem head-sharded over the ranks, one gather "
                         "per step (strong scaling, the value line); batch = every rank decodes its own config-3 "
                         "sequence (weak scaling)")
    ap.add_argument("--dist", action="store_true",
                    help="N = 1: run the multi-rank path anyway, on a world-size-1 RCCL group (init_process_group "
                         "'nccl', the per-step all_gather, its graph capture) -- the one-GPU rehearsal of the "
                         "driver's N-GPU runs")
    ap.add_argument("--eager-gather", action="store_true",
                    help="process group: time only the eager (kernel, gather) loop, no graph capture")
    ap.add_argument("--no-side-line", action="store_true",
                    help="N > 1: skip the other mode's measurement reported beside the value line")
    ap.add_argument("--rotate", type=int, default=0,
                    help="independent KV caches cycled through (0 = enough that one pass reads >= 512 MiB per rank)")
    ap.add_argument("--kv-type", default=None, choices=["q8_0", "q4_0", "f16"])
    ap.add_argument("--heads", type=int, default=None)
    ap.add_argument("--kv-heads", type=int, default=None)
    ap.add_argument("--kv-len", type=int, default=None)
    ap.add_argument("--n-q", type=int, default=None)
    ap.add_argument("--head-dim", type=int, default=None)
    ap.add_argument("--layout", default="head", choices=["head", "pos"])
    ap.add_argument("--kv-chunk", type=int, default=0)
    ap.add_argument("--spw", type=int, default=0, help="split kernel: steps per wave (0 = planner)")
    ap.add_argument("--inflight", type=int, default=0, help="split kernel: steps in flight per wave (0 = planner)")
    ap.add_argument("--no-mask", action="store_true", help="no mask tensor (diagnostics; the metric uses a mask)")
    ap.add_argument("--pf-stagger", type=int, default=2)
    ap.add_argument("--pf", type=int, default=0, help="prefill kernel: 0 auto, 1 never, 2 whenever eligible")
    ap.add_argument("--no-mq", action="store_true", help="never pick the multi-query kernel (split-KV kernel only)")
    ap.add_argument("--bd", type=int, default=0, help="batched-decode kernel: 0 auto, 1 never, 2 all-waves form, 3 role form (fattn.h FATTN_OPT_BD)")
    ap.add_argument("--bd-xcd", type=int, default=0,
                    help="batched decode workgroup order: 0 auto, 1 plain, 2 XCD-grouped (fattn.h FATTN_OPT_BD_XCD)")
    ap.add_argument("--split-xcd", type=int, default=0,
                    help="split kernel workgroup order: 0 auto, 1 plain, 2 XCD-grouped (fattn.h FATTN_OPT_SPLIT_XCD)")
    ap.add_argument("--pf-stage", type=int, default=0,
                    help="prefill over Q8_0 / Q4_0: 0 auto (staged to f16), 1 in-kernel dequantisation, 2 staged "
                         "(fattn.h FATTN_OPT_PF_STAGE)")
    ap.add_argument("--merge-in-kernel", type=int, default=0,
                    help="multi-row chunk merge: 0 second launch, 1 in-kernel when the grid is co-resident")
    ap.add_argument("--split-prio", type=int, default=0,
                    help="split kernel wave priorities: 0 staggered, 1 none, 2 staggered while issuing")
    ap.add_argument("--waves", type=int, default=0, help="split kernel waves per workgroup (4, 8, 16; 0 = planner)")
    ap.add_argument("--no-step-skip", action="store_true", help="split kernel: load and compute every step")
    ap.add_argument("--fused-merge", action="store_true",
                    help="split kernel, multi-row tiles: last-arriving workgroup merges (no second launch)")
    ap.add_argument("--mask-live", type=float, default=1.0,
                    help="diagnostics: mask positions from this fraction of N on to -inf (a padded cache)")
    ap.add_argument("--wave-merge", type=int, default=-1, help="split/dec one-row tiles: 0 per-wave merge, 1 LDS merge")
    ap.add_argument("--prefill-mask", default="zero", choices=["zero", "random", "causal", "none"],
                    help="mask of the prefill measurement (SURVEY.md §8d: zero); the random-mask form is "
                         "reported beside it")
    ap.add_argument("--prefill-kv", default="q8_0", choices=["q8_0", "q4_0", "f16"],
                    help="K/V type of the prefill measurement (the metric's is q8_0)")
    ap.add_argument("--prefill-only", action="store_true",
                    help="N=1: only the prefill measurement, as a line tools/pmc_summary.py can tag traffic with")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = OMP_NUM_THREADS, else os.cpu_count()")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prefill", action="store_true", help="skip the prefill-shape MFMA measurement")
    ap.add_argument("--no-scale-ref", action="store_true", help="N=1: skip the config-5 strong-scaling reference")
    ap.add_argument("--no-copy-peak", action="store_true", help="skip the measured copy-kernel peak")
    ap.add_argument("--dump-out", default="", help="rank 0 writes rotation 0's inputs and gathered output (.npz)")
    return ap.parse_args(argv)


def apply_options(args):
    import fattn
    opts = [(args.spw, fattn.OPT_SPLIT_STEPS), (args.inflight, fattn.OPT_SPLIT_INFLIGHT), (args.pf, fattn.OPT_PF),
            (int(args.no_mq), fattn.OPT_MQ_DISABLE), (args.split_prio, fattn.OPT_SPLIT_PRIO), (args.bd, fattn.OPT_BD), (args.bd_xcd, fattn.OPT_BD_XCD),
            (args.split_xcd, fattn.OPT_SPLIT_XCD),
            (args.pf_stage, fattn.OPT_PF_STAGE),
            (args.waves, fattn.OPT_SPLIT_WAVES)]
    fattn.set_option(fattn.OPT_SPLIT_SKIP, 1 if args.no_step_skip else 0)
    fattn.set_option(fattn.OPT_SPLIT_MERGE, 1 if args.fused_merge else 0)
    fattn.set_option(fattn.OPT_MERGE_IN_KERNEL, args.merge_in_kernel)
    for val, opt in opts:
        if val:
            fattn.set_option(opt, val)
    fattn.set_option(fattn.OPT_PF_STAGGER, args.pf_stagger)
    if args.wave_merge >= 0:
        fattn.set_option(fattn.OPT_SPLIT_WAVE_MERGE, args.wave_merge)


def shape_of(args, workload):
    """The workload's shape; explicit flags override the preset."""
    w = dict(WORKLOADS[workload])
    for k in w:
        v = getattr(args, k)
        if v is not None:
            w[k] = v
    return w


# FATTN_BENCH_REHEARSE=1: rehearse the multi-rank path on a one-GPU box -- every
# rank on cuda:0, gloo instead of RCCL, collectives staged through host memory
# (never the measured configuration: the driver's N-GPU runs use RCCL)
REHEARSE = os.environ.get("FATTN_BENCH_REHEARSE") == "1"


def _gather(x, mode="head", buf=None, out=None):
    """head: the ranks' head slices -> the full [.., H, D] output (gather_heads);
    batch: the ranks' own sequences stacked on a leading [world] axis.
    `buf` / `out`: preallocated gather and result buffers (the form a captured
    HIP graph replays); fresh tensors when None."""
    import torch
    import torch.distributed as dist
    from fattn.shard import gather_heads
    world = dist.get_world_size()
    if REHEARSE:  # gloo: staged through host memory
        y = x.cpu()
        if mode == "head":
            res = gather_heads(y)
        else:
            res = torch.empty((world,) + tuple(y.shape), dtype=y.dtype)
            dist.all_gather_into_tensor(res.view(world * y.shape[0], *y.shape[1:]), y.contiguous())
        if out is not None:
            out.copy_(res)
            return out
        return res.to(x.device)
    if mode == "head":
        return gather_heads(x, buf=buf, out=out)
    if out is None:
        out = torch.empty((world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out.view(world * x.shape[0], *x.shape[1:]), x.contiguous())
    return out


def run_decode(args, dev, shape, rank=0, world=1, mode="head", dist_on=False):
    """Time K steps of the decode workload `shape` (one FLASH_ATTN_EXT per step)
    over `world` ranks: mode "head" shards its heads (strong scaling, every rank
    a slice of one global problem), mode "batch" gives every rank a whole
    problem of its own -- its own sequence of the batch (weak scaling).
    `dist_on`: a process group exists (world > 1, or --dist at world 1): every
    timed step gathers its output over it.
    Returns the measurement dict (rank 0 holds the max over ranks)."""
    import torch
    import torch.distributed as dist
    import fattn
    from fattn.shard import head_views, shard_heads

    D, H, N, NQ = shape["head_dim"], shape["heads"], shape["kv_len"], shape["n_q"]
    Hkv = shape["kv_heads"] or H
    typ = fattn.TYPE_NAMES[shape["kv_type"]]
    rb = fattn.row_size(typ, D)
    sh = shard_heads(H, Hkv, world if mode == "head" else 1, rank if mode == "head" else 0)
    # rotation sized by bytes: the caches one rank reads over a
    # pass of the rotation exceed the 256 MiB Infinity Cache twice over, so a
    # step never finds its KV on-die from the previous pass
    R = args.rotate or max(16, -(-ROTATE_BYTES // (2 * sh.n_kv * N * rb)))
    g = torch.Generator(device=dev)
    # head: the same global problem on every rank, each reads only its slice;
    # batch: every rank its own sequence
    g.manual_seed(1234 + (rank if mode == "batch" else 0))

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
    # one mask per cache of the rotation too (config 5's 64 rows are 512 KB a step)
    masks = []
    for r in range(R):
        mask = (torch.rand((NQ, npad), generator=g, device=dev) * 2 - 1).to(torch.float16)
        if args.mask_live < 1.0:  # diagnostics: a padded cache, positions past the live fraction -inf
            mask[:, int(args.mask_live * N):] = float("-inf")
        masks.append(mask)
    mask = masks[0]
    Hl = sh.n_heads
    outs = torch.empty((R, 1, NQ, Hl, D), dtype=torch.float32, device=dev)

    qv = fattn.q_view(q)
    kv = fattn.kv_view(kv_sets[0][0], typ, D, N, Hkv, layout=args.layout)
    vv = fattn.kv_view(kv_sets[0][1], typ, D, N, Hkv, layout=args.layout)
    qs, ks, vs = head_views(qv, kv, vv, sh)  # zero-copy slice (identity at world 1)
    k_off, v_off = ks.ptr - kv.ptr, vs.ptr - vv.ptr
    att = fattn.Attention(qs, ks, vs, None if args.no_mask else fattn.mask_view(mask), outs[0], 1.0 / D ** 0.5,
                          kv_chunk=args.kv_chunk)
    kname = att.describe()

    def step(i, stream=None, ev=None):
        kvs = kv_sets[i % R]
        att.retarget(k=kvs[0].data_ptr() + k_off, v=kvs[1].data_ptr() + v_off, dst=outs[i % R].data_ptr(),
                     mask=None if args.no_mask else masks[i % R].data_ptr())
        if ev is None:
            att(stream)
        else:
            att(stream, ev[0], ev[1])

    # 1) dominant-kernel duration, eager launches with HIP events recorded by
    #    libfattn around the kernel (not part of the timed region): median
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
    kern_ms_median = statistics.median(kms)

    # 2) the kernel alone: the K steps (step i reads KV cache i % R) captured
    #    back-to-back into one HIP graph and replayed; HIP events around the
    #    replay on the launch stream give the kernel's average in-stream
    #    duration.  At world 1 this replay IS the timed job (no collective).
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
    last = (K - 1) % R  # the output buffer of the last timed step
    if dist_on:
        _gather(outs[last], mode)  # warm the communicator
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = evs[0], evs[1]
    t0 = time.perf_counter()
    hip.hipEventRecord(ev0, gs.cuda_stream)
    with torch.cuda.stream(gs):
        graph.replay()
    hip.hipEventRecord(ev1, gs.cuda_stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    hip.hipEventSynchronize(ev1)
    hip.hipEventElapsedTime(C.byref(f), ev0, ev1)
    kern_ms_avg = f.value / K
    kernel_only_elapsed = elapsed
    res = {}
    if dist_on:
        # 3) the timed job with a process group: every step is one
        #    FLASH_ATTN_EXT on the rank's slice followed by the RCCL gather over
        #    xGMI of THAT step's output (head: + the permute into [1][NQ][H][D];
        #    batch: stacked [world][1][NQ][H][D]) -- a decode layer cannot start
        #    its next step before the gathered output exists.  K gathers are
        #    timed.  Two forms: the K (kernel, all_gather, permute) triples
        #    captured in ONE HIP graph and replayed (RCCL collectives capture
        #    into the graph like kernels; the value line), and the same triples
        #    launched eagerly from Python (beside it, and the value line if the
        #    capture raises -- in the same process).
        if mode == "head":
            gbuf = torch.empty((world,) + tuple(outs[0].shape), dtype=torch.float32, device=dev)
            full = torch.empty((1, NQ, H, D), dtype=torch.float32, device=dev)
        else:
            gbuf = None
            full = torch.empty((world, 1, NQ, H, D), dtype=torch.float32, device=dev)

        def gstep(i, stream=None):
            step(i, stream)
            _gather(outs[i % R], mode, gbuf, full)

        ggraph, graph_err = None, None
        if REHEARSE or args.eager_gather:
            graph_err = "not attempted (" + ("gloo rehearsal" if REHEARSE else "--eager-gather") + ")"
        else:
            try:
                ggraph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ggraph, stream=gs):
                    for i in range(K):
                        gstep(i)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001 -- any capture failure: time the eager form instead
                graph_err = f"{type(e).__name__}: {e}"[:400]
                ggraph = None
                torch.cuda.synchronize()
            # every rank replays, or none does: a replay's collectives on some
            # ranks only would wait forever for the others (capture records
            # them without communicating, so a failed capture left no
            # collective half-done)
            ok = torch.tensor([1 if ggraph is not None else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 0 and ggraph is not None:
                graph_err = "capture failed on another rank"
                ggraph = None
            if ggraph is not None:
                with torch.cuda.stream(gs):
                    ggraph.replay()  # untimed warm replay
                torch.cuda.synchronize()
        # eager form
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(gs):
            for i in range(K):
                gstep(i, gs.cuda_stream)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        eager_elapsed = time.perf_counter() - t0
        elapsed, graph_dev_ms = eager_elapsed, float("nan")
        if ggraph is not None:
            dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            hip.hipEventRecord(ev0, gs.cuda_stream)
            with torch.cuda.stream(gs):
                ggraph.replay()
            hip.hipEventRecord(ev1, gs.cuda_stream)
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
            elapsed = time.perf_counter() - t0
            hip.hipEventSynchronize(ev1)
            hip.hipEventElapsedTime(C.byref(f), ev0, ev1)
            graph_dev_ms = f.value / K
        res.update(eager_elapsed=eager_elapsed, graph_dev_ms=graph_dev_ms, graph_err=graph_err,
                   timing="graph" if ggraph is not None else "eager")

    res.update({"kernel": kname, "kernel_ms_avg": kern_ms_avg, "kernel_ms_median": kern_ms_median,
                "elapsed": elapsed, "kernel_only_elapsed": kernel_only_elapsed})
    if args.dump_out and (rank == 0 or mode == "batch"):
        # the last step's inputs (rotation `last`) and the (gathered) output,
        # for the multi-rank parity test (tests/test_rehearsal.py checks them
        # against the oracle); batch mode: every rank its own inputs
        # (<dump>.rank<r>.npz), rank 0 the gathered outputs of all ranks
        if mode == "head":
            out0 = (full if dist_on else outs[last]).cpu().numpy()
        else:
            out0 = (full if dist_on else outs[last][None]).cpu().numpy()
        path = args.dump_out if rank == 0 else args.dump_out + f".rank{rank}.npz"
        np.savez(path, q=q.cpu().numpy(), k=kv_sets[last][0].cpu().numpy(), v=kv_sets[last][1].cpu().numpy(),
                 mask=masks[last].cpu().view(torch.int16).numpy().view(np.uint16), out=out0,
                 shape=np.array([D, NQ, H, Hkv, N, typ, world]), kernel=np.array(kname), mode=np.array(mode))
    if dist_on:
        assert tuple(full.shape) == ((1, NQ, H, D) if mode == "head" else (world, 1, NQ, H, D))
        # 3) per-step cost of the gather, and kernel + gather per step (eager),
        #    reported apart from the kernel (BASELINE.md multi-GPU rule)
        one = outs[0]
        gts, ets = [], []
        for i in range(25):
            dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            _gather(one, mode)
            torch.cuda.synchronize()
            gts.append(time.perf_counter() - t)
        for i in range(25):
            dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            step(i, stream)
            _gather(outs[i % R], mode)
            torch.cuda.synchronize()
            ets.append(time.perf_counter() - t)
        res["gather_ms_median"] = statistics.median(gts[5:]) * 1e3
        res["step_with_gather_ms_median"] = statistics.median(ets[5:]) * 1e3
        keys = ("elapsed", "kernel_ms_avg", "kernel_ms_median", "gather_ms_median", "step_with_gather_ms_median",
                "kernel_only_elapsed", "eager_elapsed", "graph_dev_ms")
        t = torch.tensor([res[k] for k in keys], dtype=torch.float64, device="cpu" if REHEARSE else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        res.update(zip(keys, (float(x) for x in t.tolist())))
    for e in evs:
        hip.hipEventDestroy(e)

    # algorithmic bytes: Q + K + V + mask + O at stored precision,
    # each once; per rank its slice plus the (replicated) mask
    mask_b = 0 if args.no_mask else NQ * N * 2
    job_bytes = (NQ * H * D * 4) * 2 + 2 * Hkv * N * rb + mask_b
    rank_bytes = (NQ * Hl * D * 4) * 2 + 2 * sh.n_kv * N * rb + mask_b
    flops = 4 * NQ * N * D * H
    if mode == "batch":  # the job: `world` sequences, one per rank
        job_bytes, flops = world * job_bytes, world * flops
    res.update(job_bytes=job_bytes, rank_bytes=rank_bytes, flops=flops, rank_flops=4 * NQ * N * D * Hl,
               workload=f"decode_{shape['kv_type']}_h{H}_hkv{Hkv}_d{D}_n{N}_q{NQ}", shard=sh, R=R, mode=mode)
    return res


def roofline(res, args, traffic=None, peaks=None):
    ach = res["rank_bytes"] / (res["kernel_ms_avg"] * 1e-3) / 1e9
    ach_tf = res["rank_flops"] / (res["kernel_ms_avg"] * 1e-3) / 1e12
    if res["rank_flops"] / res["rank_bytes"] > MFMA_F16_PEAK_TFLOPS * 1e12 / (HBM_PEAK_GBS * 1e9):
        return {"bound": "mfma", "achieved": round(ach_tf, 2), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach_tf / MFMA_F16_PEAK_TFLOPS, 4), "traffic": traffic, "kernel": res["kernel"]}
    r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": res["kernel"],
         "frac_median_kernel": round(res["rank_bytes"] / (res["kernel_ms_median"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if peaks and peaks.get("oneshot"):
        os_ = peaks["oneshot"]
        best_us = os_["us_per_launch"][os_["best"]]
        r["peak_measured_oneshot"] = round(res["rank_bytes"] / (best_us * 1e-6) / 1e9, 1)
        r["frac_of_oneshot"] = round(ach / r["peak_measured_oneshot"], 4)
        r["oneshot_probe"] = {**os_, "note": "tools/hbm_copy.hip hbm_oneshot: this launch's 256 workgroups reading "
                                             "their K and V slices once, nothing else; min of 3 x 200 launches"}
    if peaks and "copy_dwordx4" in peaks:
        r["peak_measured_copy"] = peaks["copy_dwordx4"]
        r["frac_of_measured_copy"] = round(ach / peaks["copy_dwordx4"], 4)
        r["peak_measured_read"] = peaks["read_dwordx4"]
        r["frac_of_measured_read"] = round(ach / peaks["read_dwordx4"], 4)
        r["measured_peaks"] = "tools/hbm_copy.hip: dwordx4 copy (read + write bytes) and read stream, 1 GiB, median"
    return r


def spawn_ranks(n):
    """`--gpus N` without a launcher: start N ranks through torch.distributed.run
    as a child process (nothing here has touched the GPU) and exit with its code."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and args.gpus not in (1, world):
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dist and "WORLD_SIZE" not in os.environ:
        # --dist without a launcher: a world-size-1 group of our own (nothing
        # here has touched the GPU yet)
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # a process group exists: every rank of N > 1, or --dist at N = 1 (the RCCL
    # path executed on a one-GPU box: init, the per-step all_gather, capture)
    multi = world > 1 or args.dist

    import torch
    import torch.distributed as dist
    import fattn

    apply_options(args)
    if REHEARSE:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if multi:
        if REHEARSE:
            dist.init_process_group("gloo", init_method="env://")
        else:
            dist.init_process_group("nccl", init_method="env://", device_id=dev)
    if args.prefill_only and not multi:
        # (profiling passes: the prefill launches alone)
        hip, evs = hip_events(2)
        r = prefill_measure(dev, hip, evs, args.prefill_kv, args.prefill_mask)
        print(json.dumps({"metric": METRIC + " (prefill shape)", "value": r["roofline"]["achieved"], "unit": "TFLOP/s",
                          "n_gpus": 1, "kernel_ms_avg": r["kernel_ms_avg"],
                          "config": {"workload": r["workload"], "bytes_per_step": r["bytes_per_step"],
                                     "flops_per_step": r["flops_per_step"]},
                          "roofline": {**r["roofline"], "kernel": r["kernel"]}, "source_hash": source_hash()}),
              flush=True)
        return
    mode = args.multi if multi else "head"
    workload = args.workload if args.workload != "auto" else ("config5" if mode == "head" and multi else "config3")
    shape = shape_of(args, workload)
    res = run_decode(args, dev, shape, rank, world, mode, multi)
    side = None
    if multi and not args.no_side_line:
        # the other multi-GPU reading beside the value line: head mode (the line)
        # -> the weak-scaling batch of config-3 sequences; batch -> the config-5 head shard
        other = "batch" if mode == "head" else "head"
        wl = "config3" if other == "batch" else "config5"
        side = run_decode(args, dev, shape_of(argparse.Namespace(**{k: None for k in WORKLOADS[wl]}), wl),
                          rank, world, other, multi)

    if rank == 0:
        traffic = committed_traffic(res["workload"], res["kernel"]) if not multi else None
        peaks = None if args.no_copy_peak or multi else measured_hbm_peaks()
        if not args.no_copy_peak and not multi:
            one = oneshot_ceiling(shape)
            if one:
                peaks = dict(peaks or {}, oneshot=one)
        sh = res["shard"]
        K = args.steps
        value = res["job_bytes"] * K / res["elapsed"] / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(res["elapsed"] / K * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak" if mode == "batch" else "strong",
            "vs_baseline": None,
            "dtype": "f16",
            "data": "synthetic (uniform [-1,1) Q/K/V, K/V quantised on device to ggml blocks; random f16 mask)",
            "config": {"workload": res["workload"], "heads": shape["heads"], "kv_heads": shape["kv_heads"],
                       "head_dim": shape["head_dim"], "kv_len": shape["kv_len"], "n_q": shape["n_q"],
                       "kv_type": shape["kv_type"], "kv_layout": args.layout, "kv_rotation": res["R"],
                       "parallelism": ("single_gpu" if not multi else
                                       f"batch_shard_1seq_per_rank_x{world}" if mode == "batch" else
                                       f"head_shard_{sh.n_heads}heads_per_rank_x{world}"),
                       "bytes_per_step": res["job_bytes"], "flops_per_step": res["flops"]},
            "tflops": round(res["flops"] * K / res["elapsed"] / 1e12, 4),
            "kernel_ms_avg": round(res["kernel_ms_avg"], 5),
            "kernel_ms_median": round(res["kernel_ms_median"], 5),
            "kernel_timing": "avg: HIP events around the timed graph replay on the launch stream, / steps; "
                             "median: per-launch HIP events, eager",
            "roofline": roofline(res, args, traffic, peaks),
            "source_hash": source_hash(),
        }
        if multi:
            if REHEARSE:
                line["rehearsal"] = "FATTN_BENCH_REHEARSE: all ranks on one GPU, gloo, not a measurement"
            if world == 1:
                line["world1"] = ("--dist: the multi-rank path on a world-size-1 RCCL group (one GPU): "
                                  "init_process_group('nccl'), one all_gather per step, graph capture")
            line["per_rank"] = {"heads": sh.n_heads, "kv_heads": sh.n_kv, "bytes": res["rank_bytes"],
                                "sequences": 1 if mode == "batch" else f"1/{world} of the heads"}
            line["gather"] = {"collective": "all_gather_into_tensor (RCCL over xGMI) of every step's output"
                                            + (" + permute into the ggml dst layout" if mode == "head" else "")
                                            + ", K gathers inside the timed region",
                              "gathers_timed": K,
                              "timing": res["timing"],
                              "timing_note": ("graph: the K (kernel, all_gather, permute) triples captured in one HIP "
                                              "graph, replayed, wall clock between barriers, max over ranks"
                                              if res["timing"] == "graph" else
                                              "eager: kernel, gather, permute launched from Python per step"),
                              "graph_capture_error": res["graph_err"],
                              "device_ms_per_step": (round(res["graph_dev_ms"], 5)
                                                     if res["graph_dev_ms"] == res["graph_dev_ms"] else None),
                              "wall_ms_per_step": round(res["elapsed"] / K * 1e3, 5),
                              "eager_value": round(res["job_bytes"] * K / res["eager_elapsed"] / 1e9, 2),
                              "eager_ms_per_step": round(res["eager_elapsed"] / K * 1e3, 5),
                              "per_step_gather_ms_median": round(res["gather_ms_median"], 4),
                              "per_step_kernel_plus_gather_ms_median": round(res["step_with_gather_ms_median"], 4)}
            # kernel-only scaling ("near-linear" applies to the kernel
            # part): the same K launches as one graph replay, no collective
            line["kernel_only"] = {
                "value": round(res["job_bytes"] * K / res["kernel_only_elapsed"] / 1e9, 2), "unit": "GB/s",
                "ms_per_step": round(res["kernel_only_elapsed"] / K * 1e3, 5),
                "timing": "the K launches captured in one HIP graph, replayed, wall clock max over ranks; "
                          "no gather"}
            if side is not None:
                shs = side["shard"]
                key = "weak_scaling_config3" if side["mode"] == "batch" else "head_shard_config5"
                line[key] = {
                    "workload": side["workload"], "scaling": "weak" if side["mode"] == "batch" else "strong",
                    "parallelism": (f"batch_shard_1seq_per_rank_x{world}" if side["mode"] == "batch" else
                                    f"head_shard_{shs.n_heads}heads_per_rank_x{world}"),
                    "value": round(side["job_bytes"] * K / side["elapsed"] / 1e9, 2), "unit": "GB/s",
                    "ms_per_step": round(side["elapsed"] / K * 1e3, 5), "timing": side["timing"],
                    "kernel_only_value": round(side["job_bytes"] * K / side["kernel_only_elapsed"] / 1e9, 2),
                    "kernel_ms_avg": round(side["kernel_ms_avg"], 5), "kernel": side["kernel"],
                    "per_step_gather_ms_median": round(side["gather_ms_median"], 4),
                    "per_step_kernel_plus_gather_ms_median": round(side["step_with_gather_ms_median"], 4),
                    "note": ("every rank decodes its own config-3 sequence (the N=1 line's workload), one gather of "
                             "the ranks' outputs per step; weak-scaling efficiency = value / (N * the N=1 value)"
                             if side["mode"] == "batch" else
                             "one config-5 problem (n_q 64) sliced by kv heads over the ranks, one gather per step")}
        if multi:
            print(json.dumps(line), flush=True)

    if not multi:
        if not args.no_scale_ref and workload == "config3":
            # the strong-scaling reference: config 5 (the multi-GPU workload) on this one GPU
            r5 = run_decode(args, dev, shape_of(argparse.Namespace(**{k: None for k in WORKLOADS["config5"]}),
                                                "config5"))
            line["strong_scaling_ref"] = {
                "workload": r5["workload"], "value": round(r5["job_bytes"] * args.steps / r5["elapsed"] / 1e9, 2),
                "unit": "GB/s", "ms_per_step": round(r5["elapsed"] / args.steps * 1e3, 5),
                "kernel_ms_avg": round(r5["kernel_ms_avg"], 5), "kernel": r5["kernel"],
                "note": "bench.py --gpus N runs this workload head-sharded; strong-scaling efficiency = "
                        "value(N) / (N * this value)"}
        if not args.no_scale_ref and workload == "config3":
            hip, evs = hip_events(2)
            line["config5_seq64"] = seq64_measure(dev, hip, evs)
        if not args.no_prefill and shape["n_q"] == 1:
            hip, evs = hip_events(2)
            line["prefill"] = prefill_measure(dev, hip, evs, args.prefill_kv, args.prefill_mask)
            if args.prefill_mask != "random":
                r = prefill_measure(dev, hip, evs, args.prefill_kv, "random")
                line["prefill_random_mask"] = {k: r[k] for k in ("workload", "kernel", "kernel_ms_avg", "roofline")}
            if args.prefill_kv != "f16" and not args.pf_stage:
                # beside it: the same prefill with the K/V dequantised inside the
                # kernel, tile by tile (FATTN_OPT_PF_STAGE = 1; the round-4 form)
                with fattn.options({fattn.OPT_PF_STAGE: 1}):
                    r = prefill_measure(dev, hip, evs, args.prefill_kv, args.prefill_mask)
                line["prefill_inkernel_dequant"] = {k: r[k] for k in ("workload", "kernel", "kernel_ms_avg", "roofline")}
        if not args.no_cpu_baseline and shape["n_q"] == 1:  # kernel_test.h's CPU path is one query row
            threads = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, threads)
            if "prefill" in line:
                line["prefill"]["cpu_baseline"] = cpu_baseline_prefill()
        print(json.dumps(line), flush=True)
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
