"""Per-wave phase timeline of the split kernel (diagnostic build libfattn_stamps.so,
`make stamps`).

Stamps (s_memrealtime, 100 MHz = 10 ns) per wave, g_stamps[block][16][16], see
fattn_split.h: 0 start, 1 first steps issued, 2+s data of step s in LDS (s < 8),
10 loop done, 11 waves merged, 12 partial published + drained, 14 arrival
atomic returned, 15 merger's loads in, 13 tile merged and stored.
Usage: python tools/stamps.py [--kv-type q8_0] [--waves 16] [--kv-len N] ...
"""
import argparse
import ctypes as C
import os
import sys

os.environ["FATTN_LIB"] = os.environ.get("FATTN_STAMPS_LIB") or "libfattn_stamps.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fattn  # noqa: E402

NS = 16   # stamps per wave
NWS = 16  # wave slots per block

NAMES = {0: "start", 1: "first steps issued", 10: "loop done", 11: "waves merged",
         12: "published+drained", 14: "atomic returned", 15: "merger loads in", 13: "tile merged+stored"}
# waves of <= 4 steps (stamps in LDS since round 6, stored at the kernel's end)
NAMES_SHORT = {6: "step 0 computed", 7: "step 0+nbuf issued", 8: "step 1 computed", 9: "step 1+nbuf issued"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kv-chunk", type=int, default=0)
    ap.add_argument("--kv-type", default="q8_0")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=0)
    ap.add_argument("--kv-len", type=int, default=4096)
    ap.add_argument("--n-q", type=int, default=1)
    ap.add_argument("--spw", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=0)
    ap.add_argument("--waves", type=int, default=0)
    ap.add_argument("--loaders", type=int, default=0, help="FATTN_OPT_SPLIT_LOADERS (2: loader waves)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for val, opt in ((args.spw, fattn.OPT_SPLIT_STEPS), (args.inflight, fattn.OPT_SPLIT_INFLIGHT),
                     (args.waves, fattn.OPT_SPLIT_WAVES), (args.loaders, fattn.OPT_SPLIT_LOADERS)):
        if val:
            fattn.set_option(opt, val)
    D, H, N, NQ = 128, args.heads, args.kv_len, args.n_q
    Hkv = args.kv_heads or H
    typ = fattn.TYPE_NAMES[args.kv_type]
    L = fattn.lib()
    L.fattn_debug_set_stamps.argtypes = [C.c_void_p]
    sets = []
    for r in range(8):
        pair = []
        for _ in range(2):
            x = torch.rand((Hkv * N, D), device=dev) * 2 - 1
            pair.append(fattn.quantize(x, typ).reshape(-1) if typ != fattn.TYPE_F16 else
                        x.half().view(torch.uint8).reshape(-1))
        sets.append(pair)
    q = torch.rand((1, NQ, H, D), device=dev) * 2 - 1
    npad = (N + 63) // 64 * 64
    mask = (torch.rand((NQ, npad), device=dev) * 2 - 1).half()
    out = torch.empty((1, NQ, H, D), device=dev)
    att = fattn.Attention(fattn.q_view(q), fattn.kv_view(sets[0][0], typ, D, N, Hkv),
                          fattn.kv_view(sets[0][1], typ, D, N, Hkv), fattn.mask_view(mask), out, D ** -0.5,
                          kv_chunk=args.kv_chunk)
    print(att.describe())
    L.fattn_debug_plan.argtypes = [C.c_void_p, C.c_void_p]
    g = (C.c_int * 3)()
    assert L.fattn_debug_plan(C.byref(att.p), g) == 0
    nblk = g[0] * g[1] * g[2]
    st = torch.zeros(nblk * NWS * NS, dtype=torch.int64, device=dev)
    for i in range(6):
        att.retarget(k=sets[i][0].data_ptr(), v=sets[i][1].data_ptr())
        att()
    torch.cuda.synchronize()
    assert L.fattn_debug_set_stamps(st.data_ptr()) == 0
    att.retarget(k=sets[7][0].data_ptr(), v=sets[7][1].data_ptr())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    att()
    e1.record()
    torch.cuda.synchronize()
    L.fattn_debug_set_stamps(None)
    s = st.cpu().numpy().reshape(nblk, NWS, NS).astype(np.int64)
    live = s[:, :, 0] != 0
    t0 = s[:, :, 0][live].min()
    print(f"blocks {nblk}  waves {live.sum()}  event time {e0.elapsed_time(e1) * 1e3:.1f} us  "
          f"stamp span {(s.max() - t0) * 0.01:.2f} us")
    pct = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100)) if len(a) else "   -"
    print("                              min    p10    p50    p90    max  (us since the first wave's start)")
    import re
    dsc = att.describe()
    mc, mw = re.search(r"chunk (\d+)", dsc), re.search(r"(\d+)waves", dsc)
    short = bool(mc and mw) and int(mc.group(1)) // (int(mw.group(1)) * 32) <= 4  # steps per wave <= 4
    for k in (0, 1) + tuple(range(2, 10)) + (10, 11, 12, 14, 15, 13):
        v = s[:, :, k]
        m = live & (v > 0)
        if not m.any():
            continue
        name = NAMES.get(k) or (NAMES_SHORT.get(k) if short else None) or f"data of step {k - 2} in LDS"
        print(f"{name:28s}", pct((v[m] - t0) * 0.01))
    # per block: last wave's loop done -> phases of the block's epilogue
    last_loop = np.where(live, s[:, :, 10], 0).max(axis=1)
    print("durations per block (us)     min    p10    p50    p90    max")
    for a_, b_, name in ((10, 11, "last loop done -> merged"), (11, 12, "merged -> published"),
                         (12, 14, "published -> atomic"), (14, 13, "atomic -> tile stored")):
        va = last_loop if a_ == 10 else s[:, :, a_].max(axis=1)
        vb = s[:, :, b_].max(axis=1)
        m = (va > 0) & (vb > 0)
        if m.any():
            print(f"{name:28s}", pct((vb[m] - va[m]) * 0.01))
    first_data = np.where(live & (s[:, :, 2] > 0), s[:, :, 2], np.iinfo(np.int64).max).min(axis=1)
    m = first_data < np.iinfo(np.int64).max
    print(f"{'block: first data -> last loop':28s}", pct((last_loop[m] - first_data[m]) * 0.01))


if __name__ == "__main__":
    main()
