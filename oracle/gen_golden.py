"""Generate tests/golden/ fixtures from the REFERENCE's own CPU oracle.

TEST INFRASTRUCTURE ONLY.  Runs in the build container, where
oracle/_ref/libref_utils.so is compiled from /root/reference/src/utils.h
(oracle/Makefile).  The fixtures are data: inputs (or the glibc rand() recipe
that regenerates them) and the reference's outputs.

  kernel_test_cfg1.npz      BASELINE config 1: kernel_test.h call pattern
                            (srand(1), fill Q,K,V,mask, kernel_test.h:45-61)
                            at H=1, D=64, N=128 -- full inputs + output.
  kernel_test_default.npz   kernel_test.h defaults (32 q / 8 kv heads, D=128,
                            kv_size=512) -- output only; inputs regenerate
                            from srand(1).
  kernel_test_q8_0.npz      same call pattern, H=4, D=128, N=256, but K and V
                            pass through ggml Q8_0 (restated: fattn_oracle.c)
                            before the reference's mulmat/softmax -- output only.
  kat_misc_flash_attn.json  the hand-written known-answer test of
                            src/misc/flash-attn.cu:202-295 (2 heads, d=3, seq=4).

Usage: python oracle/gen_golden.py   (writes tests/golden/)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import oracle as orc  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def kernel_test_inputs(D, H, Hkv, N, impl):
    """kernel_test.h:45-48: srand unset (glibc seed 1), fill order Q, K, V, mask."""
    orc.srand(1, impl)
    q = orc.random(D * H, impl)
    k = orc.random(D * N * Hkv, impl)
    v = orc.random(D * N * Hkv, impl)
    m = orc.random(N, impl)
    return q, k, v, m


def main():
    assert orc.ref_available(), "oracle/_ref/libref_utils.so missing: run `make oracle` in the build container"
    os.makedirs(OUT, exist_ok=True)

    # config 1
    D, H, Hkv, N = 64, 1, 1, 128
    q, k, v, m = kernel_test_inputs(D, H, Hkv, N, "ref")
    out = orc.kernel_test_cpu(q, k, v, m, N, D, H, Hkv, impl="ref")
    np.savez_compressed(os.path.join(OUT, "kernel_test_cfg1.npz"), query=q, key=k, value=v, mask=m, out=out,
                        meta=np.array([D, H, Hkv, N]))

    # kernel_test defaults
    D, H, Hkv, N = 128, 32, 8, 512
    q, k, v, m = kernel_test_inputs(D, H, Hkv, N, "ref")
    out = orc.kernel_test_cpu(q, k, v, m, N, D, H, Hkv, impl="ref")
    np.savez_compressed(os.path.join(OUT, "kernel_test_default.npz"), out=out, meta=np.array([D, H, Hkv, N]),
                        q_head=q[:16], k_head=k[:16], v_head=v[:16], m_head=m[:16])

    # Q8_0 K/V through the reference's attention arithmetic
    D, H, Hkv, N = 128, 4, 4, 256
    q, k, v, m = kernel_test_inputs(D, H, Hkv, N, "ref")
    kq = orc.dequantize(orc.quantize(k.reshape(-1, D), orc.TYPE_Q8_0), orc.TYPE_Q8_0, D).reshape(-1)
    vq = orc.dequantize(orc.quantize(v.reshape(-1, D), orc.TYPE_Q8_0), orc.TYPE_Q8_0, D).reshape(-1)
    out = orc.kernel_test_cpu(q, kq, vq, m, N, D, H, Hkv, impl="ref")
    np.savez_compressed(os.path.join(OUT, "kernel_test_q8_0.npz"), out=out, meta=np.array([D, H, Hkv, N]))

    # known-answer test, src/misc/flash-attn.cu:202-295 (values transcribed as data)
    kat = {
        "source": "src/misc/flash-attn.cu:202-295",
        "d_head": 3, "seq_len": 4, "num_heads": 2, "scale": "1/sqrt(3)",
        "query": [2, 4, 2, 4, 2, 1, 4, 1, 3, 4, 2, 2, 2, 1, 1, 4, 2, 1, 1, 1, 3, 4, 2, 1],
        "key": [2, 4, 2, 4, 2, 1, 4, 2, 3, 1, 2, 1, 3, 1, 3, 4, 2, 1, 1, 1, 2, 4, 3, 1],
        "value_transposed": [2, 4, 2, 1, 2, 1, 4, 2, 1, 4, 2, 3, 1, 4, 2, 1, 2, 1, 1, 2, 1, 4, 3, 3],
        "expected": [2.0457, 2.4446, 1.3050, 2.4594, 3.2287, 2.4192, 2.0603, 3.8987, 2.0551, 2.1756, 3.6809,
                     2.1481, 1.8984, 1.6943, 2.9636, 1.7022, 1.7658, 3.1875, 1.2656, 1.8836, 1.5731, 1.7022,
                     1.7658, 3.1875],
        "layout": "query/key [head][seq][d]; value [head][d][seq]; expected [head][seq][d]",
    }
    with open(os.path.join(OUT, "kat_misc_flash_attn.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
