"""ISA audit of the untracked inline-asm register loads (round-3 verdict item 7),
on the CPU: tools/isa_hazard_check.py over the -save-temps ISA of every
translation unit of libfattn.so (`make isa`, the library's own flags).

* The shipped tree is clean: on every control-flow path no instruction touches
  the destination VGPRs of an untracked load before its reg_fence marker, and
  every asm register load is tagged.
* The audited ISA IS the shipped code: each function's instruction sequence
  equals the disassembly of the gfx950 code objects inside libfattn.so.
* The audit catches the hazard: a probe kernel with a deliberately injected
  early store and an early register copy of a pending load is flagged, the
  correct form of the same kernel is not.
* Its second audit (asm wait states): an asm v_add_f32 that reads a v_exp_f32
  result hipcc placed right before it is flagged; with the pad inside the asm
  it is not.  The shipped ISA has none.  Likewise the third (an XDL result read
  by asm) and the fourth (a v_readfirstlane'd descriptor word read by an asm
  VMEM instruction within 5 wait states).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_hazard_check as ihc  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
LIB = os.path.join(ROOT, "ggml-cuda-experiments_amd", "lib", "libfattn.so")
CSRC = os.path.join(ROOT, "ggml-cuda-experiments_amd", "csrc")


def _isa_files():
    """build/isa/*.s, rebuilt by make when a source is newer (make's own rule)."""
    r = subprocess.run(["make", "-C", ROOT, "-j8", "isa"], capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-3000:]
    units = sorted(f[:-4] for f in os.listdir(CSRC) if f.endswith(".hip"))
    files = [os.path.join(ROOT, "build", "isa", u + ".s") for u in units]
    assert all(os.path.exists(f) for f in files), files
    return files


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_shipped_isa_has_no_untracked_load_hazards(capsys):
    files = _isa_files()
    assert os.path.exists(LIB), "libfattn.so not built"
    rc = ihc.main(["--same-as", LIB] + files)
    out = capsys.readouterr().out
    print(out[-4000:])
    assert rc == 0, out[-4000:]
    assert "0 hazards" in out and "0 mismatches" in out and "0 asm wait-state hazards" in out
    # the audit saw the loads it is about (the split kernel's Q / mask words)
    n_loads = int(out.split("functions in")[1].split(":")[1].split("untracked")[0])
    assert n_loads > 0


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_audit_catches_injected_early_touch(tmp_path, capsys):
    src = os.path.join(ROOT, "tests", "hip", "isa_hazard_probe.hip")
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/include", "-c", src,
                        "-save-temps", "-o", "probe.o"], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    s = str(tmp_path / "isa_hazard_probe-hip-amdgcn-amd-amdhsa-gfx950.s")
    funcs = ihc.parse_functions(s)
    by = {}
    for name, body in funcs.items():
        findings, loads, rets = ihc.check_function(name, body)
        key = next(k for k in ("probe_clean", "probe_early_store", "probe_early_copy", "probe_trans_asm_use",
                               "probe_trans_asm_padded", "probe_xdl_asm_read_padded", "probe_xdl_asm_read",
                               "probe_xdl_vgpr_read_padded", "probe_xdl_vgpr_read",
                               "probe_sgpr_vmem_padded", "probe_sgpr_vmem")
                   if k in name)
        by[key] = (findings, loads, rets, ihc.check_wait_states(name, body) + ihc.check_xdl_asm_reads(name, body) +
                   ihc.check_sgpr_vmem(name, body))
    assert set(by) == {"probe_clean", "probe_early_store", "probe_early_copy", "probe_trans_asm_use",
                       "probe_trans_asm_padded", "probe_xdl_asm_read", "probe_xdl_asm_read_padded",
                       "probe_xdl_vgpr_read", "probe_xdl_vgpr_read_padded", "probe_sgpr_vmem", "probe_sgpr_vmem_padded"}
    # the fourth audit: a descriptor word fresh from v_readfirstlane read by an
    # asm LDS-DMA after s_nop 0 is flagged; behind the helper's s_nop 4 it is not
    sw = by["probe_sgpr_vmem"][3]
    assert sw and sw[0][0].mnem.startswith("v_readfirstlane") and sw[0][1].mnem.startswith("buffer_load"), sw
    assert by["probe_sgpr_vmem_padded"][3] == []
    # the third audit: an asm accumulator read right behind an XDL MFMA (across
    # the branch) is flagged; with 24 wait states of s_nop it is not
    xw = by["probe_xdl_asm_read"][3]
    assert xw and xw[0][0].mnem.startswith("v_mfma") and xw[0][1].mnem.startswith("v_accvgpr_read"), xw
    assert by["probe_xdl_asm_read_padded"][3] == []
    # ... and hipcc's read right behind an asm MFMA chain into VGPRs is flagged
    # (once: the chain's own second step is not), not behind the chain's pad
    vw = by["probe_xdl_vgpr_read"][3]
    assert len(vw) == 1 and vw[0][0].in_asm and vw[0][0].ops.endswith(vw[0][0].ops.split(",")[0].strip()), vw
    assert not vw[0][1].in_asm and vw[0][1].mnem.startswith("v_"), vw
    assert by["probe_xdl_vgpr_read_padded"][3] == []
    ws = by["probe_trans_asm_use"][3]
    assert ws and ws[0][0].mnem.startswith("v_exp") and ws[0][1].mnem.startswith("v_add"), ws
    assert by["probe_trans_asm_padded"][3] == []
    for k in ("probe_clean", "probe_early_store", "probe_early_copy"):
        assert by[k][3] == [], k
    assert by["probe_clean"][0] == [] and by["probe_clean"][1] == 1 and by["probe_clean"][2] == 1
    store = by["probe_early_store"][0]
    assert store and any(ins.mnem.startswith("global_store") for ins, _, _ in store), store
    copy = by["probe_early_copy"][0]
    assert copy and any(ins.mnem.startswith("v_mov") for ins, _, _ in copy), copy
    assert ihc.main([s]) == 1  # the command line reports them too
