"""test_llama over real dumps (src/flash-matrix.cu:67-339): load
<dir>/<prefix>-{q,k,v,mask,qkv}-<n>.tensor, run FLASH_ATTN_EXT through libfattn,
print the max abs difference against the qkv dump (and against the CPU oracle
restatement when --oracle).

usage: python tools/run_tensors.py DIR [--prefix fa-cuda] [--n 256]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ggml-cuda-experiments_amd"), ROOT]

import numpy as np  # noqa: E402

from fattn import tensor_io as tio  # noqa: E402
from fattn.dumps import attention_from_dumps  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--prefix", default="fa-cuda")
ap.add_argument("--n", default="256")
ap.add_argument("--scale", type=float, default=None)
args = ap.parse_args()
path = lambda w: os.path.join(args.dir, f"{args.prefix}-{w}-{args.n}.tensor")
t = {w: tio.load_tensor(path(w)) for w in ("q", "k", "v", "mask")}
for w, x in t.items():
    print(f"Tensor: {x.name:>15s} type {x.type} ne {list(x.ne)}")
got = attention_from_dumps(t["q"], t["k"], t["v"], t["mask"], args.scale)
if os.path.exists(path("qkv")):
    ref = np.asarray(tio.load_tensor(path("qkv")).data, dtype=np.float32).reshape(got.shape)
    print(f"max abs diff vs qkv dump: {np.abs(got - ref).max():.6g}")
else:
    print("no qkv dump; out[0, 0, :4] =", got.reshape(-1)[:4])
