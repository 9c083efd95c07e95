import ctypes as C, os, sys
os.environ["FATTN_LIB"] = "libfattn_stamps.so"
sys.path[:0] = ["/root/repo/ggml-cuda-experiments_amd", "/root/repo"]
import numpy as np, torch, fattn
dev = torch.device("cuda:0")
D, H, N = 128, 32, 4096
typ = fattn.TYPE_Q8_0
L = fattn.lib(); L.fattn_debug_set_stamps.argtypes = [C.c_void_p]
k = fattn.quantize(torch.rand((H * N, D), device=dev) * 2 - 1, typ).reshape(-1)
v = fattn.quantize(torch.rand((H * N, D), device=dev) * 2 - 1, typ).reshape(-1)
q = torch.rand((1, 1, H, D), device=dev) * 2 - 1
mask = (torch.rand((1, N), device=dev) * 2 - 1).half()
out = torch.empty((1, 1, H, D), device=dev)
att = fattn.Attention(fattn.q_view(q), fattn.kv_view(k, typ, D, N, H), fattn.kv_view(v, typ, D, N, H), fattn.mask_view(mask), out, D ** -0.5, kv_chunk=int(sys.argv[1]))
for it in range(3):
    st = torch.zeros(65536 * 4 * 16, dtype=torch.int64, device=dev)
    assert L.fattn_debug_set_stamps(st.data_ptr()) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); att(); e1.record(); torch.cuda.synchronize()
    s = st.cpu().numpy().reshape(-1, 4, 16)
    nb = (s[:, 0, 0] != 0).sum()
    s = s[:nb]
    last = s[:, 0, 13] > 0
    print("  slot9 (chunk+1, tag, seen):", [(int(x) >> 40, (int(x) >> 32) & 0xff, int(x) & 0xffffffff) for x in s[last, 0, 9][:6]])
    print(f"it {it} time {e0.elapsed_time(e1)*1e3:.0f} us  blocks {nb} last {last.sum()}  ml-spin max {s[last,0,14].max()} fetch-spin max {s[last,0,15].max()}  slow mc {sorted(set((s[last,0,11][s[last,0,11] > 999999] - 1000000).tolist()))[:10]}")
    ws = att.workspace.view(torch.int64)[:8 * 32 * 4].view(-1, 32)[:, 0].cpu().numpy()
    print("  arrival words (epoch<<32|count):", [(int(x) >> 32, int(x) & 0xffffffff) for x in ws[:4]])
# dump the tagged partial units of tile 0
g = (C.c_int * 3)()
L.fattn_debug_plan.argtypes = [C.c_void_p, C.c_void_p]
L.fattn_debug_plan(C.byref(att.p), g)
nch, ny, nz = g[0], g[1], g[2]
arrive_bytes = nz * ny * 256
part = att.workspace[arrive_bytes:].view(torch.int32).cpu().numpy()
UPR = D // 2 + 1
for c in range(nch):
    base = ((0 * nch + c) * 16 + 0) * UPR * 4
    print("tile0 chunk", c, "unit0", part[base:base + 4], "unitML", part[base + (D // 2) * 4: base + (D // 2) * 4 + 4])
