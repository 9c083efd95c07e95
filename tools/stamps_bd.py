"""Per-wave phase timeline of the batched-decode kernel (diagnostic build
libfattn_stamps.so, `make stamps`; never the product library).

Stamps (s_memrealtime, 100 MHz = 10 ns) per wave, g_stamps[block][16][16],
fattn_bd.h: 0 start, 1 prologue issued, 2 Q ready, 3 + 2s tile s landed, 4 + 2s
tile s computed (s < 4), 14 / 15 tile 0 past barrier 1 / 2, 11 loop done,
12 states parked, 13 stores drained.
--form bdp (fattn_bdp.h, FATTN_OPT_BD = 3): 0 start, 1 prologue issued, 2
prologue done, 3 + s past tile s's barrier, 7 + s tile s's work done (compute
waves 0-3: tile s computed; build waves 4-7: raw s + 1 dequantised and raw
s + 2 landed), s < 4; 11 loop done, 12 states parked, 13 partials stored --
printed per role.
Usage: python tools/stamps_bd.py [--form bd|bdp] [--heads 4] [--kv-len 4096] [--n-q 64] [--kv-chunk 0]
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

NS, NWS = 16, 16
NAMES = {0: "start", 1: "prologue issued", 2: "Q ready", 14: "tile 0 barrier 1", 15: "tile 0 V image",
         11: "loop done", 12: "states parked", 13: "stores drained"}
for s_ in range(4):
    NAMES[3 + 2 * s_] = f"tile {s_} landed"
    NAMES[4 + 2 * s_] = f"tile {s_} computed"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kv-chunk", type=int, default=0)
    ap.add_argument("--kv-type", default="q8_0")
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--kv-len", type=int, default=4096)
    ap.add_argument("--n-q", type=int, default=64)
    ap.add_argument("--form", default="bd", choices=["bd", "bdp"])
    args = ap.parse_args()
    fattn.set_option(fattn.OPT_BD, 2 if args.form == "bd" else 3)
    dev = torch.device("cuda:0")
    D, H, N, NQ = 128, args.heads, args.kv_len, args.n_q
    typ = fattn.TYPE_NAMES[args.kv_type]
    L = fattn.lib()
    L.fattn_debug_set_stamps.argtypes = [C.c_void_p]
    L.fattn_debug_plan.argtypes = [C.c_void_p, C.c_void_p]
    R = 24
    sets = [[fattn.quantize(torch.rand((H * N, D), device=dev) * 2 - 1, typ).reshape(-1) for _ in range(2)]
            for _ in range(R)]
    q = torch.rand((1, NQ, H, D), device=dev) * 2 - 1
    npad = (N + 63) // 64 * 64
    mask = (torch.rand((NQ, npad), device=dev) * 2 - 1).half()
    out = torch.empty((1, NQ, H, D), device=dev)
    att = fattn.Attention(fattn.q_view(q), fattn.kv_view(sets[0][0], typ, D, N, H),
                          fattn.kv_view(sets[0][1], typ, D, N, H), fattn.mask_view(mask), out, D ** -0.5,
                          kv_chunk=args.kv_chunk)
    print(att.describe())
    g = (C.c_int * 3)()
    assert L.fattn_debug_plan(C.byref(att.p), g) == 0
    nblk = g[0] * g[1] * g[2]
    st = torch.zeros(nblk * NWS * NS, dtype=torch.int64, device=dev)
    for i in range(R - 1):
        att.retarget(k=sets[i][0].data_ptr(), v=sets[i][1].data_ptr())
        att()
    torch.cuda.synchronize()
    assert L.fattn_debug_set_stamps(st.data_ptr()) == 0
    att.retarget(k=sets[R - 1][0].data_ptr(), v=sets[R - 1][1].data_ptr())
    att()
    torch.cuda.synchronize()
    L.fattn_debug_set_stamps(None)
    s = st.cpu().numpy().reshape(nblk, NWS, NS).astype(np.int64)
    live = s[:, :, 0] != 0
    t0 = s[:, :, 0][live].min()
    print(f"blocks {nblk}  waves {live.sum()}  stamp span {(s.max() - t0) * 0.01:.2f} us")
    pct = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100)) if len(a) else "   -"
    print("                              min    p10    p50    p90    max  (us since the first wave's start)")
    if args.form == "bd":
        for k in (0, 1, 2, 3, 14, 15, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13):
            v = s[:, :, k]
            m = live & (v > 0)
            if m.any():
                print(f"{NAMES[k]:28s}", pct((v[m] - t0) * 0.01))
        return
    names = {0: "start", 1: "prologue issued", 2: "prologue done", 11: "loop done", 12: "states parked",
             13: "partials stored", 14: "tile 2: raw issue begins", 15: "tile 2: raw 2+nRaw issued"}
    for s_ in range(4):
        names[3 + s_] = f"past tile {s_} barrier"
        names[7 + s_] = f"tile {s_} work done"
    for role, ws in (("compute waves 0-3", slice(0, 4)), ("build waves 4-7", slice(4, 8))):
        print(f"-- {role}")
        for k in (0, 1, 2, 3, 7, 4, 8, 5, 14, 15, 9, 6, 10, 11, 12, 13):
            v = s[:, ws, k]
            m = live[:, ws] & (v > 0)
            if m.any():
                print(f"{names[k]:28s}", pct((v[m] - t0) * 0.01))
    print("per-wave durations (us)      min    p10    p50    p90    max")
    for a_, b_, name in ((0, 1, "start -> prologue issued"), (1, 2, "-> Q ready"), (2, 3, "Q ready -> tile 0 landed"),
                         (3, 14, "-> barrier 1"), (14, 15, "-> V image (barrier 2)"), (15, 4, "-> tile 0 computed"),
                         (4, 5, "tile 0 computed -> tile 1 landed"), (5, 6, "-> tile 1 computed"),
                         (11, 12, "loop done -> parked"), (12, 13, "parked -> stores drained")):
        m = live & (s[:, :, a_] > 0) & (s[:, :, b_] > 0)
        if m.any():
            print(f"{name:28s}", pct((s[:, :, b_][m] - s[:, :, a_][m]) * 0.01))


if __name__ == "__main__":
    main()
