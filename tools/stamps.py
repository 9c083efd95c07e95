"""Per-wave phase timeline of the split kernel (diagnostic build libfattn_stamps.so).

Stamps (s_memrealtime, 100 MHz = 10 ns) per wave:
 0 start  1 first LDS-DMA issued  2 first step's data in LDS  3 loop done
 4 4-wave merge barrier passed  5 end (partial or output stored)
Usage: python tools/stamps.py [--kv-chunk N] [--kv-type q8_0] ...
"""
import argparse
import ctypes as C
import os
import sys

os.environ["FATTN_LIB"] = "libfattn_nocompute.so" if "--nocompute" in sys.argv else "libfattn_stamps.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import fattn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kv-chunk", type=int, default=0)
    ap.add_argument("--kv-type", default="q8_0")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--kv-heads", type=int, default=0)
    ap.add_argument("--kv-len", type=int, default=4096)
    ap.add_argument("--n-q", type=int, default=1)
    ap.add_argument("--nocompute", action="store_true", help="memory-only diagnostic build")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
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
    st = torch.zeros(nblk * 4 * 8, dtype=torch.int64, device=dev)
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
    s = st.cpu().numpy().reshape(-1, 8).astype(np.int64)
    s = s[s[:, 0] != 0]
    t0 = s[:, 0].min()
    rel = lambda k: (s[:, k] - t0) * 0.01  # us
    print(f"waves {len(s)}  event time {e0.elapsed_time(e1) * 1e3:.1f} us  "
          f"stamp span {(s[:, :6].max() - t0) * 0.01:.2f} us")
    pct = lambda a: " ".join(f"{np.percentile(a, p):6.2f}" for p in (0, 10, 50, 90, 100))
    print("                          min    p10    p50    p90    max  (us)")
    print("start                    ", pct(rel(0)))
    print("dma issued   (1-0)       ", pct((s[:, 1] - s[:, 0]) * 0.01))
    print("data arrival (2)         ", pct(rel(2)[s[:, 2] > 0]))
    print("wait data    (2-1)       ", pct(((s[:, 2] - s[:, 1]) * 0.01)[s[:, 2] > 0]))
    print("loop         (3-2)       ", pct(((s[:, 3] - s[:, 2]) * 0.01)[s[:, 2] > 0]))
    print("loop done    (3)         ", pct(rel(3)))
    print("merge barrier(4-3)       ", pct((s[:, 4] - s[:, 3]) * 0.01))
    print("store       (5-4)       ", pct((s[:, 5] - s[:, 4]) * 0.01))
    print("end          (5)         ", pct(rel(5)))


if __name__ == "__main__":
    main()
