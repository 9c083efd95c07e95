"""Debug probe: the batched-decode plan on masked problems (causal, tail,
neginf blocks) against the oracle -- which rows come out NaN or wrong.
Test infrastructure (imports the oracle through tests/problems.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "ggml-cuda-experiments_amd"))
import fattn  # noqa: E402
from gpu_util import upload, views  # noqa: E402
from problems import make_problem, attn_rel_err  # noqa: E402


def run(p, kv_chunk=0):
    import torch
    t = upload(p, "cuda")
    att = fattn.Attention(*views(p, t), t["dst"], p.scale, kv_chunk=kv_chunk)
    d = att.describe()
    att()
    torch.cuda.synchronize()
    return t["dst"].cpu().numpy(), d


cases = [
    (dict(D=128, NQ=1024, H=8, N=1024, kv_type="q8_0", mask="random", seed=43), 0),
    (dict(D=128, NQ=1024, H=8, N=1024, kv_type="q8_0", mask="causal", seed=43), 1024),
    (dict(D=128, NQ=128, H=1, N=1024, kv_type="q8_0", mask="causal", seed=43), 0),
    (dict(D=128, NQ=64, H=1, N=512, kv_type="q8_0", mask="causal", seed=43), 512),
    (dict(D=128, NQ=64, H=1, N=512, kv_type="q8_0", mask="random", seed=43), 512),
    (dict(D=128, NQ=64, H=1, N=512, kv_type="q8_0", mask="none", seed=43), 512),
    (dict(D=128, NQ=64, H=1, N=512, kv_type="q8_0", mask="neginf_blocks", seed=43), 512),
    (dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0", mask="neginf_blocks", seed=43), 1024),
]
fattn.set_option(fattn.OPT_PF, 1)
for c, kc in cases:
    p = make_problem(**c)
    got, d = run(p, kc)
    ref = p.oracle()
    g = got.reshape(-1, p.D)
    r = ref.reshape(-1, p.D)
    gn = np.isnan(g).any(1)
    rn = np.isnan(r).any(1)
    bad = np.nonzero(gn != rn)[0]
    print(c, "|", d)
    print("  nan rows got", int(gn.sum()), "ref", int(rn.sum()), "mismatched", len(bad), "first", bad[:8].tolist(),
          "(row = (q * H + h))")
    ok = ~(gn | rn)
    if ok.any():
        err = np.abs(g[ok] - r[ok]).max(1) / np.maximum(np.abs(r[ok]).max(1), 1e-30)
        print("  max rel err over finite rows %.3g" % err.max())
    sys.stdout.flush()
