"""Per-wave phase timeline of the split kernel (diagnostic build libfattn_stamps.so).

Stamps (s_memrealtime, 100 MHz = 10 ns) per wave, see fattn_split.h:
 0 start  1 first steps issued  2+s data of step s in LDS (s < 8)
 10 loop done  11 4-wave merge done  12 partial published / output stored
 13 tile merge done (last workgroup of a tile only)
Usage: python tools/stamps.py [--kv-chunk N] [--kv-type q8_0] [--nocompute] ...
"""
import argparse
import ctypes as C
import os
import sys

os.environ["FATTN_LIB"] = os.environ.get("FATTN_STAMPS_LIB") or ("libfattn_nocompute.so" if "--nocompute" in sys.argv else
                           "libfattn_stamps_nomem.so" if "--nomem" in sys.argv else "libfattn_stamps.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fattn  # noqa: E402

NS = 16


def att_chunks(att):
    """n_chunks of the plan: workspace = epochs + tagged partials (fattn_api.hip)."""
    ws = fattn.workspace_size(att.p)
    if ws == 0:
        return 1
    q = att.p.q
    D, NQ, H = q.ne[0], q.ne[1], q.ne[2]
    Hkv = att.p.k.ne[2]
    r = H // Hkv
    R = min(r, 16)
    QPT = 16 // R
    Y = Hkv * ((r + R - 1) // R) * ((NQ + QPT - 1) // QPT)
    S = q.ne[3]
    per_chunk = S * Y * 16 * (D // 2 + 1) * 16
    return (ws - S * Y * 256) // per_chunk


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
    ap.add_argument("--nocompute", action="store_true", help="memory-only diagnostic build")
    ap.add_argument("--nomem", action="store_true", help="compute-only diagnostic build")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.spw:
        fattn.set_option(fattn.OPT_SPLIT_STEPS, args.spw)
    if args.inflight:
        fattn.set_option(fattn.OPT_SPLIT_INFLIGHT, args.inflight)
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
    nblk = 65536 * 4
    st = torch.zeros(nblk * 4 * NS, dtype=torch.int64, device=dev)
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
    s = st.cpu().numpy().reshape(-1, NS).astype(np.int64)
    s = s[s[:, 0] != 0]
    t0 = s[:, 0].min()
    us = lambda k: (s[:, k] - t0) * 0.01
    have = lambda k: s[:, k] > 0
    print(f"waves {len(s)}  event time {e0.elapsed_time(e1) * 1e3:.1f} us  "
          f"stamp span {(s.max() - t0) * 0.01:.2f} us")
    pct = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100)) if len(a) else "   -"
    print("                          min    p10    p50    p90    max  (us since first wave start)")
    print("start                    ", pct(us(0)))
    print("steps issued             ", pct(us(1)))
    for k in range(8):
        if have(2 + k).any():
            print(f"data step {k}              ", pct(us(2 + k)[have(2 + k)]))
    print("loop done                ", pct(us(10)))
    print("merge done               ", pct(us(11)[have(11)]))
    print("published/stored         ", pct(us(12)[have(12)]))
    print("tile merge done (last wg)", pct(us(13)[have(13)]))
    # chunk hand-off, per tile (grid x = chunk; block-major stamp layout)
    L.fattn_debug_plan.argtypes = [C.c_void_p, C.c_void_p]
    g = (C.c_int * 3)()
    assert L.fattn_debug_plan(C.byref(att.p), g) == 0
    nch, ny, nz = g[0], g[1], g[2]
    if nch > 1:
        blk = st.cpu().numpy().reshape(-1, 4, NS)[: nch * ny * nz].astype(np.int64)
        blk = blk.reshape(-1, nch, 4, NS)
        wmax = lambda k: (blk[..., k].max(axis=2) - t0) * 0.01   # latest wave of each block
        last = blk[..., 0, 13] > 0                                 # the merging block of each tile
        t11, t12, t13 = wmax(11), wmax(12), wmax(13)
        print(f"tiles {len(blk)} x {nch} chunks")
        print("4-wave merge done, all    ", pct(t11.reshape(-1)))
        print("published+atomic, all     ", pct(t12.reshape(-1)))
        print("  (12-11) drain+atomic    ", pct((t12 - t11).reshape(-1)))
        print("last wg: merge done (13)  ", pct(t13[last]))
        print("last wg: 13-12 combine    ", pct((t13 - t12)[last]))
        t14, t15 = wmax(14), wmax(15)
        print("  14-12 loads RT          ", pct((t14 - t12)[last]))
        print("  15-14 weights+barrier   ", pct((t15 - t14)[last]))
        print("  13-15 fold+sum+store    ", pct((t13 - t15)[last]))
        print("last wg: 12 - max others11", pct(np.array([t12[i][last[i]].max() - np.delete(t11[i], np.where(last[i])[0]).max()
                                                          for i in range(len(blk))])))
    # per-step compute: gap between consecutive step arrivals
    for k in range(1, 8):
        m = have(2 + k) & have(1 + k)
        if m.any():
            print(f"step {k - 1}->{k} gap          ", pct((s[m, 2 + k] - s[m, 1 + k]) * 0.01))


if __name__ == "__main__":
    main()
