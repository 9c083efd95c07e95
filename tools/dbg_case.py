"""Debug helper: run one parity problem on the GPU and print where it differs."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

from gpu_util import run_gpu  # noqa: E402
from problems import attn_rel_err, make_problem  # noqa: E402

cases = [
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0", layout="head", seed=30),
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0", layout="head", seed=30, mask="none"),
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q8_0", layout="pos", seed=30),
    dict(D=128, NQ=1, H=4, N=256, kv_type="q8_0", layout="head", seed=30),
    dict(D=128, NQ=1, H=4, N=128, kv_type="q8_0", layout="head", seed=30),
    dict(D=128, NQ=1, H=1, N=32, kv_type="q8_0", layout="head", seed=30),
    dict(D=128, NQ=1, H=32, N=4096, kv_type="q4_0", layout="head", seed=30),
    dict(D=128, NQ=1, H=32, N=2048, kv_type="f16", layout="head", seed=30),
]
for c in cases:
    for chunk in (0, 100000):
        p = make_problem(**c)
        got, ref = run_gpu(p, kv_chunk=chunk), p.oracle()
        e = attn_rel_err(got, ref)
        g = got.reshape(-1, p.D)
        r = ref.reshape(-1, p.D)
        nan_rows = np.where(np.isnan(g).any(axis=1))[0]
        bad = np.where(np.abs(g - r).max(axis=1) > 1e-3 * np.abs(r).max(axis=1))[0]
        print(c, "chunk", chunk, "err", e, "nan rows", nan_rows[:8], "bad rows", bad[:8], "n_bad", len(bad))
        if len(bad):
            i = bad[0]
            print("   got", g[i, :6], "\n   ref", r[i, :6])
