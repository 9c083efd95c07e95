"""Debug helper: multi-query kernel cases at 64 rows per wave; print where they differ."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import fattn  # noqa: E402
from gpu_util import run_gpu  # noqa: E402
from problems import attn_rel_err, make_problem  # noqa: E402

cases = [
    dict(D=128, kv_type="q8_0", NQ=300, H=2, Hkv=2, N=256, mask="causal"),
    dict(D=128, kv_type="q8_0", NQ=300, H=2, Hkv=2, N=256, mask="none"),
    dict(D=128, kv_type="q8_0", NQ=256, H=2, Hkv=2, N=256, mask="random"),
    dict(D=128, kv_type="q8_0", NQ=256, H=1, Hkv=1, N=32, mask="none"),
]
for rpw in (16, 64):
    fattn.set_option(fattn.OPT_MQ_ROWS_PER_WAVE, rpw)
    for c in cases:
        for chunk in (0, 100000):
            p = make_problem(seed=5, **c)
            got, ref = run_gpu(p, kv_chunk=chunk), p.oracle()
            e = attn_rel_err(got, ref)
            g = got.reshape(-1, p.D)
            r = ref.reshape(-1, p.D)
            bad = np.where(~(np.abs(g - r) <= 1e-3 * np.nan_to_num(np.abs(r)).max(axis=1, keepdims=True)).all(axis=1)
                           & ~(np.isnan(g).all(axis=1) & np.isnan(r).all(axis=1)))[0]
            print("rpw", rpw, c, "chunk", chunk, "err", e, "n_bad", len(bad), "bad rows", bad[:12], flush=True)
            if len(bad):
                i = bad[0]
                print("   got", g[i, :6], "\n   ref", r[i, :6])
                badc = np.where(np.abs(g[i] - r[i]) > 1e-3)[0]
                print("   bad cols", badc[:20], len(badc))
