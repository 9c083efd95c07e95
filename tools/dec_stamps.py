"""Phase timeline of fattn_dec_kernel (diagnostic build lib/libfattn_stamps.so,
-DFATTN_STAMPS; the product library executes no stamp).

Stamps (s_memrealtime, 100 MHz = 10 ns) per wave, [block][8 waves][16]:
 0 entry
 loader waves:  2 first AH steps issued, 3 first step landed (FULL set), 4 last FULL set
 compute waves: 2 Q landed, 3 first FULL seen, 5 last step's FULL seen, 6 loop done,
                10 partial stored + drained, 11 arrival atomic returned,
                12 merger: partial loads landed, 13 merger: dst stored
Usage: python tools/dec_stamps.py [--kv-type q8_0] [--heads 32] [--kv-heads 0] [--kv-len 4096] [--n-q 1]
       [--dec-compute 4] [--dec-loaders 2] [--diag 0]
"""
import argparse
import ctypes as C
import os
import sys

os.environ["FATTN_LIB"] = os.environ.get("FATTN_STAMPS_LIB", "libfattn_stamps.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fattn  # noqa: E402

NS = 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kv-type", default="q8_0")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=0)
    ap.add_argument("--kv-len", type=int, default=4096)
    ap.add_argument("--n-q", type=int, default=1)
    ap.add_argument("--dec-compute", type=int, default=0)
    ap.add_argument("--dec-loaders", type=int, default=0)
    ap.add_argument("--diag", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    fattn.set_option(fattn.OPT_DEC, 2)
    if args.dec_compute:
        fattn.set_option(fattn.OPT_DEC_COMPUTE, args.dec_compute)
    if args.dec_loaders:
        fattn.set_option(fattn.OPT_DEC_LOADERS, args.dec_loaders)
    if args.diag:
        fattn.set_option(fattn.OPT_DEC_DIAG, args.diag)
    D, H, N, NQ = 128, args.heads, args.kv_len, args.n_q
    Hkv = args.kv_heads or H
    typ = fattn.TYPE_NAMES[args.kv_type]
    L = fattn.lib()
    L.fattn_debug_set_stamps.argtypes = [C.c_void_p]
    sets = []
    for r in range(12):
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
                          fattn.kv_view(sets[0][1], typ, D, N, Hkv), fattn.mask_view(mask), out, D ** -0.5)
    print(att.describe())
    nblk = 65536
    st = torch.zeros(nblk * 8 * NS, dtype=torch.int64, device=dev)
    for i in range(10):
        att.retarget(k=sets[i][0].data_ptr(), v=sets[i][1].data_ptr())
        att()
    torch.cuda.synchronize()
    assert L.fattn_debug_set_stamps(st.data_ptr()) == 0
    att.retarget(k=sets[11][0].data_ptr(), v=sets[11][1].data_ptr())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    att()
    e1.record()
    torch.cuda.synchronize()
    L.fattn_debug_set_stamps(None)
    s = st.cpu().numpy().reshape(-1, 8, NS).astype(np.int64)
    s = s[s[:, 0, 0] != 0]
    t0 = s[:, :, 0][s[:, :, 0] > 0].min()
    ncw = args.dec_compute or 4
    comp, load = s[:, :ncw], s[:, ncw:]
    load = load[load[:, :, 0] > 0].reshape(len(s), -1, NS) if load.size else load
    print(f"blocks {len(s)}  event time {e0.elapsed_time(e1) * 1e3:.1f} us  stamp span {(s.max() - t0) * 0.01:.2f} us")

    def pct(x):
        x = x[x > 0]
        if not len(x):
            return "   -"
        x = (x - t0) * 0.01
        return " ".join(f"{np.percentile(x, p):6.2f}" for p in (0, 10, 50, 90, 100))

    print("                               min    p10    p50    p90    max  (us since the first wave's entry)")
    print("entry                      ", pct(s[:, :, 0].reshape(-1)))
    print("loader: first steps issued ", pct(load[:, :, 2].reshape(-1)))
    print("loader: first step landed  ", pct(load[:, :, 3].reshape(-1)))
    print("loader: last step landed   ", pct(load[:, :, 4].reshape(-1)))
    print("compute: Q landed          ", pct(comp[:, :, 2].reshape(-1)))
    print("compute: first FULL seen   ", pct(comp[:, :, 3].reshape(-1)))
    print("compute: last FULL seen    ", pct(comp[:, :, 5].reshape(-1)))
    print("compute: loop done         ", pct(comp[:, :, 6].reshape(-1)))
    print("partial stored+drained     ", pct(comp[:, :, 10].reshape(-1)))
    print("arrival atomic returned    ", pct(comp[:, :, 11].reshape(-1)))
    print("merger: partial loads in   ", pct(comp[:, :, 12].reshape(-1)))
    print("merger: dst stored         ", pct(comp[:, :, 13].reshape(-1)))
    d = lambda a, b: ((a - b) * 0.01)[(a > 0) & (b > 0)]
    q = lambda x: " ".join(f"{np.percentile(x, p):6.2f}" for p in (0, 10, 50, 90, 100)) if len(x) else "   -"
    print("durations                      min    p10    p50    p90    max")
    print("loop done - last FULL (last step compute)", q(d(comp[:, :, 6], comp[:, :, 5]).reshape(-1)))
    print("drain (10 - 6)                           ", q(d(comp[:, :, 10], comp[:, :, 6]).reshape(-1)))
    print("atomic (11 - 10)                         ", q(d(comp[:, :, 11], comp[:, :, 10]).reshape(-1)))
    print("merger loads (12 - 11)                   ", q(d(comp[:, :, 12], comp[:, :, 11]).reshape(-1)))
    print("merger finish (13 - 12)                  ", q(d(comp[:, :, 13], comp[:, :, 12]).reshape(-1)))


if __name__ == "__main__":
    main()
