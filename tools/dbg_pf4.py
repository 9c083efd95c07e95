#!/usr/bin/env python3
"""Diagnostic: fattn_pf4_kernel against fattn_pf_kernel on small f16 prefills,
row by row (which waves / row blocks / lanes differ)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ggml-cuda-experiments_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import fattn
    from gpu_util import upload, views
    from problems import make_problem
    for case in [dict(kv_type="f16", NQ=256, H=1, Hkv=1, N=64, mask="none"),
                 dict(kv_type="f16", NQ=256, H=1, Hkv=1, N=64, mask="random"),
                 dict(kv_type="f16", NQ=256, H=1, Hkv=1, N=256, mask="none"),
                 dict(kv_type="f16", NQ=256, H=1, Hkv=1, N=256, mask="random")]:
        p = make_problem(seed=5, **case)
        ref = p.oracle()[0, :, 0, :]
        outs = {}
        fattn.set_option(fattn.OPT_PF, 2)
        for form in (1, 2, 3, 4, 5):
            fattn.set_option(fattn.OPT_PF_FORM, form)
            t = upload(p)
            att = fattn.Attention(*views(p, t), t["dst"], p.scale)
            att()
            torch.cuda.synchronize()
            outs[form] = t["dst"].cpu().numpy()[0, :, 0, :]
        fattn.reset_options()
        print("case", case)
        for form in (1, 2, 3, 4, 5):
            o = outs[form]
            err = np.abs(o - ref).max(axis=1) / np.abs(ref).max(axis=1)
            bad = np.nonzero(err > 1e-3)[0]
            print(f"  form {form}: rows bad {len(bad)}/256", end="")
            if len(bad):
                ratio = np.median(o[bad] / ref[bad], axis=1)
                print(f"  first {bad[:12].tolist()} ratio {np.round(ratio[:8], 3).tolist()}", end="")
                for w in range(4):
                    for rb in range(2):
                        rows = np.arange(64 * w + 32 * rb, 64 * w + 32 * rb + 32)
                        nb = np.isin(rows, bad).sum()
                        if nb:
                            print(f" | w{w}rb{rb}:{nb}", end="")
            print()


if __name__ == "__main__":
    main()
