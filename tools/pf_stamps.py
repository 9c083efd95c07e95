"""Per-phase shader-clock cycles of the prefill kernel (diagnostic build
libfattn_stamps.so, -DFATTN_STAMPS): summed over tiles per wave, printed as
the mean cycles per tile for waves 0-3 and 4-7.
Usage: python tools/pf_stamps.py [--no-mask] [--n-q 4096] [--kv-type q8_0]"""
import argparse
import ctypes as C
import os
import sys

os.environ.setdefault("FATTN_LIB", "libfattn_stamps.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import fattn  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--no-mask", action="store_true")
ap.add_argument("--mask-zero", action="store_true", help="an all-zero mask (the bench's prefill)")
ap.add_argument("--n-q", type=int, default=4096)
ap.add_argument("--kv-len", type=int, default=4096)
ap.add_argument("--heads", type=int, default=32)
ap.add_argument("--kv-type", default="q8_0")
ap.add_argument("--form", type=int, default=0, help="FATTN_OPT_PF_FORM (0: the planner's body)")
args = ap.parse_args()
dev = torch.device("cuda:0")
fattn.set_option(fattn.OPT_PF_FORM, args.form)
D, H, N, NQ = 128, args.heads, args.kv_len, args.n_q
typ = fattn.TYPE_NAMES[args.kv_type]
if args.kv_type == "f16":
    k = (torch.rand((H * N, D), device=dev) * 2 - 1).half().reshape(-1)
    v = (torch.rand((H * N, D), device=dev) * 2 - 1).half().reshape(-1)
else:
    k = fattn.quantize(torch.rand((H * N, D), device=dev) * 2 - 1, typ).reshape(-1)
    v = fattn.quantize(torch.rand((H * N, D), device=dev) * 2 - 1, typ).reshape(-1)
q = torch.rand((1, NQ, H, D), device=dev) * 2 - 1
mask = (torch.rand((NQ, (N + 63) // 64 * 64), device=dev) * 2 - 1).half()
if args.mask_zero:
    mask.zero_()
out = torch.empty((1, NQ, H, D), device=dev)
att = fattn.Attention(fattn.q_view(q), fattn.kv_view(k, typ, D, N, H), fattn.kv_view(v, typ, D, N, H),
                      None if args.no_mask else fattn.mask_view(mask), out, D ** -0.5)
L = fattn.lib()
L.fattn_debug_set_stamps.argtypes = [C.c_void_p]
st = torch.zeros(65536 * 8 * 16, dtype=torch.int64, device=dev)
for _ in range(3):
    att()
torch.cuda.synchronize()
assert L.fattn_debug_set_stamps(st.data_ptr()) == 0
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
att()
e1.record()
torch.cuda.synchronize()
L.fattn_debug_set_stamps(None)
s = st.cpu().numpy().reshape(-1, 8, 16)
s = s[s[:, 0, 8] > 0]
nt = s[:, :, 8].astype(np.float64)
names = ["wait+barrier", "dma issue", "dequant", "S^T mfma", "softmax", "O^T mfma", "-", "loop tail"]
pf4 = "fattn_pf4_kernel" in att.describe()
if pf4:  # the pipelined one-wave-per-SIMD body (fattn_pf4.h SCHED 2): 4 waves
    names = ["A wait", "A steps", "A tail", "B barrier", "B head", "B steps", "B tail", "between tiles"]
print(att.describe())
print(f"workgroups {len(s)}  event {e0.elapsed_time(e1) * 1e3:.1f} us  (cycles per tile, mean)")
for half, sl in (("waves 0-3", slice(0, 4)),) + ((("waves 4-7", slice(4, 8)),) if not pf4 else ()):
    per = s[:, sl, :8].astype(np.float64) / nt[:, sl, None]
    tot = per.sum(axis=2).mean()
    print(f"{half}: total {tot:8.0f}  " + "  ".join(f"{n} {per[..., i].mean():6.0f}" for i, n in enumerate(names) if n != "-"))
if pf4 and (s[:, 0, 12] > 0).any():
    # workgroup timeline (fattn_pf4_kernel, slots 9-15): shader clocks of entry /
    # loop start / loop end / exit, real-time (100 MHz) entry / exit, HW_ID | XCC_ID
    w = s[:, :4, :].astype(np.float64)
    pro = (w[:, :, 10] - w[:, :, 9]).mean()
    loop = (w[:, :, 11] - w[:, :, 10]).mean()
    epi = (w[:, :, 12] - w[:, :, 11]).mean()
    life = (w[:, :, 12] - w[:, :, 9]).mean()
    rt = (w[:, :, 14] - w[:, :, 13])
    mhz = ((w[:, :, 12] - w[:, :, 9]) / np.maximum(rt, 1)).mean() * 100.0
    print(f"workgroup lifetime {life:.0f} cyc: prologue {pro:.0f}  loop {loop:.0f}  epilogue {epi:.0f}; "
          f"shader clock ~{mhz:.0f} MHz; lifetime {rt.mean() / 100:.1f} us real time")
    r0 = w[:, 0, 13].min()
    ent = (w[:, 0, 13] - r0) / 100.0
    ex = (w[:, :, 14].max(axis=1) - r0) / 100.0
    print(f"entry times (us from the first): quantiles 0/25/50/75/100 % "
          + " ".join(f"{x:.1f}" for x in np.percentile(ent, [0, 25, 50, 75, 100]))
          + f"; last exit {ex.max():.1f} us")
    hw = s[:, 0, 15].astype(np.uint64)
    cu = ((hw >> np.uint64(8)) & np.uint64(0xF)) | (((hw >> np.uint64(13)) & np.uint64(0x7)) << np.uint64(4)) \
        | (((hw >> np.uint64(12)) & np.uint64(1)) << np.uint64(7)) | ((hw >> np.uint64(32)) & np.uint64(0xF)) << np.uint64(8)
    uq, cnt = np.unique(cu, return_counts=True)
    print(f"distinct (xcc, se, sh, cu) {len(uq)}; workgroups per CU: "
          + " ".join(f"{c}x{n}" for c, n in zip(*np.unique(cnt, return_counts=True))))
    # per-CU busy span vs the kernel span
    busy = {}
    for i, c in enumerate(cu):
        busy.setdefault(int(c), []).append((w[i, :, 13].min(), w[i, :, 14].max()))
    gaps = [sorted(v)[1][0] - sorted(v)[0][1] for v in busy.values() if len(v) >= 2]
    if gaps:
        print(f"gap between a CU's 1st exit and 2nd entry: mean {np.mean(gaps) / 100:.2f} us "
              f"max {np.max(gaps) / 100:.2f}")
