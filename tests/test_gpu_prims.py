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


@pytest.mark.parametrize("use_buffer", [0, 1, 2], ids=["global_load_lds", "buffer_load_lds", "buffer_load_lds_oob"])
@pytest.mark.parametrize("nact", [64, 16])
def test_lds_dma_partial_exec(dev, use_buffer, nact):
    """LDS-DMA writes lane-linear 16-B pieces at base + 16*lane; with a partial
    EXEC mask only the active lanes' pieces may change (fattn_split.h issues a
    partial last instruction for 136-B Q8_0 rows).  "oob": all 64 lanes issue,
    the others with an offset past the descriptor: they fetch nothing but
    write ZEROS to their LDS pieces (so OOB rows/positions read back as 0)."""
    import torch
    L = C.CDLL(LIB)
    src = torch.arange(4096, dtype=torch.int32, device=dev).to(torch.uint8)
    out = torch.zeros(2048, dtype=torch.uint8, device=dev)
    assert L.prims_dma_partial(C.c_void_p(src.data_ptr()), C.c_void_p(out.data_ptr()), nact, use_buffer) == 0
    o = out.cpu().numpy()
    s = src.cpu().numpy()
    exp = np.full(2048, 0xAB, np.uint8)
    exp[256:256 + 16 * nact] = s[:16 * nact]
    if use_buffer == 2:
        exp[256 + 16 * nact:256 + 16 * 64] = 0
    diff = np.where(o != exp)[0]
    if len(diff):
        print(f"\n{len(diff)} bytes differ; first at {diff[:8]}; got {o[diff[:8]]} exp {exp[diff[:8]]}")
    assert len(diff) == 0
