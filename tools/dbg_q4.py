import sys; sys.path[:0]=['.','ggml-cuda-experiments_amd','tests']
import numpy as np, torch, fattn
from oracle import oracle as orc
rng = np.random.default_rng(2)
x = (rng.standard_normal((512, 128)) * np.exp2(rng.uniform(-10, 10, (512, 1)))).astype(np.float32)
x[3] = 0.0; x[7, :32] = 1.0
ref = orc.quantize(x, 2).reshape(-1, 18)
got = fattn.quantize(torch.from_numpy(x).cuda(), 2).cpu().numpy().reshape(-1, 18)
bad = np.where((ref != got).any(1))[0]
print("bad blocks", len(bad), bad[:20])
for b in bad[:4]:
    xb = x.reshape(-1, 32)[b]
    print("block", b, "ref", ref[b], "\ngot", got[b])
    print("x", xb)
