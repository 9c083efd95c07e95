"""GPU: semantics of the gfx950 cross-lane primitives the kernels rely on."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
LIB = os.path.join(os.path.dirname(__file__), "_build", "libprims.so")


def test_permlane_swap_group_reductions(dev):
    import torch
    L = C.CDLL(LIB)
    x = torch.tensor(np.random.default_rng(0).standard_normal(64).astype(np.float32), device=dev)
    out = torch.zeros(6 * 64, device=dev)
    assert L.prims_permlane(C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr())) == 0
    o = out.cpu().numpy().reshape(6, 64)
    xs = x.cpu().numpy()
    src = lambda v: [int(np.argmin(np.abs(xs - e))) for e in v]
    print("\nr16[0] src lanes", src(o[0]))
    print("r16[1] src lanes", src(o[1]))
    print("r32[0] src lanes", src(o[2]))
    print("r32[1] src lanes", src(o[3]))
    lanes = np.arange(64)
    grp = [xs[[l & 15, (l & 15) + 16, (l & 15) + 32, (l & 15) + 48]] for l in lanes]
    np.testing.assert_array_equal(o[4], np.array([g.max() for g in grp], np.float32))
    ref_sum = np.array([(np.float32(g[0] + g[1]) + np.float32(g[2] + g[3])) for g in grp], np.float32)
    np.testing.assert_allclose(o[5], ref_sum, rtol=1e-6)
