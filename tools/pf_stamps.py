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
