#!/usr/bin/env python3
"""Diagnostic: the oracle error of the second-launch merges with f16 vs f32
chunk partials (FATTN_OPT_PART_F16) on config 5, its shards and a large-|v|
case -- how much of the 1e-3 bar the f16 rounding of O/l uses."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), os.path.join(ROOT, "tests"), ROOT]
import fattn  # noqa: E402
from gpu_util import run_gpu  # noqa: E402
from problems import attn_elem_err, attn_rel_err, make_problem  # noqa: E402

CASES = {
    "config5": dict(D=128, NQ=64, H=32, N=4096, kv_type="q8_0"),
    "config5_s8": dict(D=128, NQ=64, H=4, N=4096, kv_type="q8_0"),
    "config5_extreme": dict(D=128, NQ=64, H=8, N=4096, kv_type="q8_0", extreme=True),
    "gqa_f16_d256": dict(D=256, NQ=4, H=8, Hkv=2, N=2048, kv_type="f16"),
}
for name, case in CASES.items():
    p = make_problem(seed=5, **case)
    ref = p.oracle()
    errs = []
    for mode in (1, 2):
        with fattn.options({fattn.OPT_PART_F16: mode}):
            got = run_gpu(p)
        errs.append((attn_rel_err(got, ref), attn_elem_err(got, ref)))
    print(f"{name:18s} f32 partials rel {errs[0][0]:.3e} elem {errs[0][1]:.3f} | "
          f"f16 partials rel {errs[1][0]:.3e} elem {errs[1][1]:.3f}", flush=True)
