#!/usr/bin/env python3
"""ISA audit of the untracked inline-asm register loads (round-3 verdict item 7).

hipcc does not model the memory operations inside an `asm volatile` statement:
the VGPR destination of an asm VMEM load counts as written at `;;#ASMEND`, so
the compiler may read, copy, spill or reuse that register before the data has
landed -- silently wrong results.  The product keeps exactly one kind of such
load (ggml-cuda-experiments_amd/csrc/fattn_split.h `ld_buf_untracked<TAG>`:
the split kernel's Q and mask-word prefetch, left untracked so that waiting for
it does not drain the LDS-DMA issued behind it); every other hand-off load is a
compiler-tracked builtin.  Each untracked load carries the asm comment
`UNTRACKED(tag)`; the caller waits for it with a counted `s_waitcnt` and then
passes every result through `reg_fence<TAG>` (fattn_common.h), whose asm
comment `RETIRED(tag) <registers>` marks the point from which it may be used.

This tool proves, on the compiler's own output (the `-save-temps` ISA of every
shipped translation unit, `make isa`), that on EVERY control-flow path from an
untracked load no instruction names any of its destination VGPRs -- as source
or destination, VALU, copy, spill or address -- before its RETIRED marker (or
an `s_waitcnt vmcnt(0)`).  The wait itself precedes the fence in the source,
and volatile asm statements keep their order.
May-analysis over the CFG of each kernel (labels and s_branch / s_cbranch_*
edges), union at joins, to a fixpoint.  It also rejects any asm VMEM load with
a VGPR destination that carries no UNTRACKED tag.

Second audit (round 5): VALU wait states the compiler cannot see.  hipcc's
hazard recognizer pads its own instructions, not the text of an asm
statement, so an asm instruction that reads the result of a transcendental
(v_exp/v_log/v_rcp/v_rsq/v_sqrt/v_sin/v_cos: 1 wait state before a VALU use),
or a v_permlane*_swap that reads a VALU result (2 wait states), must carry its
own padding.  Every such producer/consumer pair where either side is inside an
asm statement is checked along straight-line code (a block and its
fall-through), counting one wait state per instruction between and N + 1 per
`s_nop N` (fattn_pf4.h's row sums once read a stale exponential this way).

Third audit (round 6): an XDL MFMA's result read by an asm instruction (e.g.
fattn_pf4.h's scale_acc16 `v_accvgpr_read` of O in the rare rescale branch)
needs the MFMA's passes + 3 wait states, which only a hand-placed `s_nop` can
give it: every path from each MFMA, across branches, is walked up to 40
instructions for an asm read of its destination registers.

`--same-as LIB.so` additionally checks that the audited ISA is the shipped
code: every function's instruction sequence (alignment nops aside) equals the
disassembly of the gfx950 code objects inside the library.

Fourth audit (round 6): a VALU instruction that writes an SGPR (v_readfirstlane,
v_readlane, a VOP3 carry-out or compare mask) followed by a VMEM instruction
that reads that SGPR (descriptor, soffset, base) needs 5 wait states; hipcc
pads its own VMEM instructions, not an asm one, so every asm VMEM
instruction's SGPR operands are checked against the VALU writes before it
(its block and the straight-line block falling into it).  (The LDS-DMA
helper's "{m0}" form once opened with s_nop 0 only: a readfirstlane'd
descriptor word two instructions ahead made multi-chunk decodes read
garbage.)

Usage: isa_hazard_check.py [--same-as lib.so] file.s [file.s ...]
Exit 0 = clean; 1 = hazards (listed); 2 = usage / parse problem.
"""
from __future__ import annotations

import argparse
import os
import re
import struct
import subprocess
import sys
from collections import defaultdict

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
VMEM_PREFIX = ("buffer_", "global_", "flat_", "scratch_", "tbuffer_")
BRANCH_RE = re.compile(r"^s_(c?branch\w*)\s+(\.L\w+|\S+)")


def vregs(text: str) -> set[int]:
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


class Insn:
    __slots__ = ("line", "mnem", "ops", "comment", "in_asm", "text")

    def __init__(self, line, mnem, ops, comment, in_asm, text):
        self.line, self.mnem, self.ops, self.comment, self.in_asm, self.text = line, mnem, ops, comment, in_asm, text


def parse_functions(path: str):
    """{function name: (list of ('label', name) | ('insn', Insn))} from a .s file."""
    funcs = {}
    cur = None
    body = None
    in_asm = False
    prev_type = None
    with open(path) as f:
        for ln, raw in enumerate(f, 1):
            line = raw.rstrip("\n")
            st = line.strip()
            if not st:
                continue
            if cur is None:
                m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
                if m and not m.group(1).startswith(".") and prev_type == m.group(1):
                    cur, body = m.group(1), []
                    in_asm = False
                    continue
                mt = re.match(r"^\s*\.type\s+([\w.$]+),@function", line)
                if mt:
                    prev_type = mt.group(1)
                continue
            if st.startswith(".Lfunc_end"):
                funcs[cur] = body
                cur = None
                prev_type = None
                continue
            if st == ";;#ASMSTART":
                in_asm = True
                continue
            if st == ";;#ASMEND":
                in_asm = False
                continue
            if st.startswith(";") or st.startswith("//"):
                if in_asm and "RETIRED(" in st:  # reg_fence<TAG>'s marker: a pseudo-instruction
                    body.append(("insn", Insn(ln, "RETIRED", st.split(")", 1)[1], st, True, st)))
                continue
            m = re.match(r"^(\.L\w+):", st)
            if m:
                body.append(("label", m.group(1)))
                continue
            if st.startswith("."):
                continue  # directives
            code, _, comment = st.partition(";")
            code = code.strip()
            if not code:
                continue
            parts = code.split(None, 1)
            body.append(("insn", Insn(ln, parts[0], parts[1] if len(parts) > 1 else "", comment, in_asm, code)))
    return funcs


def is_vmem(mn: str) -> bool:
    return mn.startswith(VMEM_PREFIX)


def vgpr_dest_load(ins: Insn) -> bool:
    """A VMEM instruction that writes VGPRs: a load (not LDS-DMA) or a returning atomic."""
    mn = ins.mnem
    if not is_vmem(mn):
        return False
    if "_load_lds" in mn or re.search(r"\blds\b", ins.ops):
        return False
    if "_load" in mn:
        return True
    if "_atomic" in mn and re.search(r"\b(sc0|glc)\b", ins.ops):
        return True
    return False


def dest_and_rest(ins: Insn):
    """(dest vregs, the other vregs named) of a VGPR-destination VMEM instruction."""
    first, _, rest = ins.ops.partition(",")
    return vregs(first), vregs(rest)


def build_blocks(body):
    """Basic blocks: list of (label or None, [Insn]), successor indices."""
    blocks = []
    cur_label, cur = None, []
    for kind, x in body:
        if kind == "label":
            if cur or cur_label is not None:
                blocks.append((cur_label, cur))
            cur_label, cur = x, []
        else:
            cur.append(x)
            if x.mnem in ("s_endpgm", "s_setpc_b64") or x.mnem.startswith("s_branch") or \
                    x.mnem.startswith("s_cbranch"):
                blocks.append((cur_label, cur))
                cur_label, cur = None, []
    if cur or cur_label is not None:
        blocks.append((cur_label, cur))
    index = {lab: i for i, (lab, _) in enumerate(blocks) if lab is not None}
    succ = []
    for i, (_, insns) in enumerate(blocks):
        s = []
        last = insns[-1] if insns else None
        if last is not None and last.mnem in ("s_endpgm", "s_setpc_b64"):
            pass
        elif last is not None and (last.mnem.startswith("s_branch") or last.mnem.startswith("s_cbranch")):
            tgt = last.ops.split()[0].rstrip(",") if last.ops else ""
            if tgt not in index:
                raise ValueError(f"branch target {tgt!r} not found (line {last.line})")
            s.append(index[tgt])
            if last.mnem.startswith("s_cbranch") and i + 1 < len(blocks):
                s.append(i + 1)
        elif i + 1 < len(blocks):
            s.append(i + 1)
        succ.append(s)
    return blocks, succ


def transfer(insns, state, report):
    """Run a block: state = {vreg: (tag, load line)} of pending untracked loads."""
    st = dict(state)
    for ins in insns:
        mn = ins.mnem
        untracked = ins.in_asm and vgpr_dest_load(ins)
        if untracked:
            dst, rest = dest_and_rest(ins)
            for r in rest & st.keys():
                report(ins, r, st[r])
            m = re.search(r"UNTRACKED\((\d+)\)", ins.comment)
            if not m:
                report(ins, None, ("untagged asm load", ins.line))
                tag = -1
            else:
                tag = int(m.group(1))
            for r in dst:
                st[r] = (tag, ins.line)
            continue
        if mn == "RETIRED":
            mask = int(re.search(r"RETIRED\((\d+)\)", ins.comment).group(1))
            st = {k: v for k, v in st.items() if not (v[0] > 0 and v[0] & mask)}
            continue
        named = vregs(ins.ops)
        hit = named & st.keys()
        for r in sorted(hit):
            report(ins, r, st[r])
        if mn == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ins.ops)
            if m and int(m.group(1)) == 0:
                st.clear()
        elif mn in ("s_swappc_b64", "s_call_b64"):
            report(ins, None, ("call inside a kernel with untracked state", ins.line)) if st else None
    return st


def check_function(name, body):
    blocks, succ = build_blocks(body)
    n = len(blocks)
    inp = [None] * n
    inp[0] = {}
    findings = {}

    def report(ins, reg, info):
        key = (ins.line, reg)
        if key not in findings:
            findings[key] = (ins, reg, info)

    work = [0]
    seen_out = [None] * n
    while work:
        i = work.pop()
        out = transfer(blocks[i][1], inp[i], report)
        if seen_out[i] == out:
            continue
        seen_out[i] = out
        for j in succ[i]:
            merged = dict(inp[j]) if inp[j] is not None else {}
            changed = inp[j] is None
            for r, v in out.items():
                if r not in merged:
                    merged[r] = v
                    changed = True
            if changed:
                inp[j] = merged
                work.append(j)
    loads = sum(1 for _, b in blocks for ins in b if ins.in_asm and vgpr_dest_load(ins))
    retires = sum(1 for _, b in blocks for ins in b if ins.mnem == "RETIRED")
    return list(findings.values()), loads, retires


# ------------------------------------------------------------------ wait states around asm

TRANS_RE = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)(_legacy)?_f(16|32)(_e32|_e64)?$")


def valu_dest_and_srcs(ins: Insn):
    """(dest vregs, source vregs) of a VALU instruction (first operand = dest)."""
    first, _, rest = ins.ops.partition(",")
    return vregs(first), vregs(rest)


def required_waits(prod: Insn, cons: Insn) -> int:
    """Wait states `cons` needs after `prod` when it reads prod's result (0: none)."""
    if not prod.mnem.startswith("v_") or prod.mnem.startswith("v_mfma") or prod.mnem.startswith("v_accvgpr"):
        return 0
    pd, _ = valu_dest_and_srcs(prod)
    if cons.mnem.startswith("v_permlane") and "swap" in cons.mnem:
        # both operands are read (and written)
        if pd & vregs(cons.ops):
            return 2
        return 0
    if TRANS_RE.match(prod.mnem) and cons.mnem.startswith("v_") and not TRANS_RE.match(cons.mnem):
        _, cs = valu_dest_and_srcs(cons)
        if pd & cs:
            return 1
    return 0


AREG = re.compile(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b")


def aregs(text: str) -> set[int]:
    out = set()
    for m in AREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def xdl_waits(mnem: str) -> int:
    """Wait states a VALU read (v_accvgpr_read included) of an XDL MFMA's result
    needs on gfx950: the pads hipcc itself places after a builtin MFMA read by
    the next VALU (32x32x16 f16 / bf16 12 states, 16x16x32 8: measured on
    hipcc's gfx950 output); other shapes by their passes + 3, the larger form
    of each (32x32 16 passes, 16x16 8, 4x4 4)."""
    # gfx950's own pads (hipcc on a builtin MFMA read by the next VALU):
    # 32x32x16 f16 / bf16 s_nop 11, 16x16x32 f16 / bf16 s_nop 7
    if re.search(r"32x32x16_(f16|bf16)$", mnem):
        return 12
    if re.search(r"16x16x32_(f16|bf16)$", mnem):
        return 8
    if "32x32" in mnem:
        return 19
    if "16x16" in mnem:
        return 11
    return 7


def accumulate_chain(prod: Insn, cons: Insn) -> bool:
    """cons is the next step of prod's accumulate chain: the same MFMA taking
    prod's whole destination as srcC and writing it back (0 wait states)."""
    if cons.mnem != prod.mnem:
        return False
    po = [o.strip() for o in prod.ops.split(",")]
    co = [o.strip() for o in cons.ops.split(",")]
    return len(po) >= 4 and len(co) >= 4 and co[0] == po[0] and co[3] == po[0]


def check_xdl_asm_reads(name, body, horizon=40):
    """XDL MFMA result -> an asm instruction reading it (round-6 advisor item),
    or an asm MFMA's result -> any vector reader: hipcc pads the wait states of
    its own VALU reads of its own MFMAs' results only (fattn_pf4.h's scale_acc16
    reads O's AGPRs in the rare rescale branch, behind a hand-placed s_nop pad;
    the lean body's S^T chains are asm MFMAs into VGPRs that hipcc's code reads).  Every path from
    each MFMA, through branches, up to `horizon` instructions or a
    redefinition, is walked; an asm instruction that names one of the MFMA's
    destination registers before the wait states have passed is a finding."""
    blocks, succ = build_blocks(body)
    findings = []
    for bi, (_, insns) in enumerate(blocks):
        for a, prod in enumerate(insns):
            if not prod.mnem.startswith("v_mfma"):
                continue
            first, _, _ = prod.ops.partition(",")
            dv, da = vregs(first), aregs(first)
            need = xdl_waits(prod.mnem)
            # depth-first over (block, start index, waits so far, steps so far)
            stack = [(bi, a + 1, 0, 0)]
            seen = set()
            while stack:
                b, k, waits, steps = stack.pop()
                if (b, k, waits) in seen:
                    continue
                seen.add((b, k, waits))
                ins_list = blocks[b][1]
                stopped = False
                while k < len(ins_list):
                    cons = ins_list[k]
                    if waits >= need or steps >= horizon:
                        stopped = True
                        break
                    if (cons.in_asm or prod.in_asm) and cons.mnem.startswith(("v_", "ds_", "buffer_", "global_")):
                        if accumulate_chain(prod, cons):
                            stopped = True  # the chain's next step redefines the registers
                            break
                        if (vregs(cons.ops) & dv) or (aregs(cons.ops) & da):
                            findings.append((prod, cons, need, waits))
                            stopped = True
                            break
                    if cons.mnem == "s_nop":
                        try:
                            waits += int(cons.ops.split()[0], 0) + 1
                        except ValueError:
                            waits += 1
                    else:
                        waits += 1
                    steps += 1
                    k += 1
                if not stopped:
                    for nb in succ[b]:
                        stack.append((nb, 0, waits, steps))
    return findings


def check_wait_states(name, body):
    """Producer/consumer pairs with an asm side that lack their wait states."""
    blocks, succ = build_blocks(body)
    findings = []
    for i, (_, insns) in enumerate(blocks):
        seq = list(insns)
        # straight-line continuation into the fall-through block
        if insns and not (insns[-1].mnem.startswith("s_branch") or insns[-1].mnem == "s_endpgm") \
                and i + 1 < len(blocks):
            seq += blocks[i + 1][1][:4]
        for a, prod in enumerate(insns):
            if not prod.mnem.startswith("v_"):
                continue
            waits = 0
            for cons in seq[a + 1:a + 6]:
                need = required_waits(prod, cons)
                if need and waits < need and (prod.in_asm or cons.in_asm):
                    findings.append((prod, cons, need, waits))
                if cons.mnem == "s_nop":
                    try:
                        waits += int(cons.ops.split()[0], 0) + 1
                    except ValueError:
                        waits += 1
                else:
                    waits += 1
                if waits >= 2:
                    break
    return findings


SREG = re.compile(r"\bs\[(\d+):(\d+)\]|\bs(\d+)\b")
SDST2 = ("v_add_co_", "v_sub_co_", "v_subrev_co_", "v_addc_co_", "v_subb_co_", "v_subbrev_co_", "v_mad_u64_u32",
         "v_mad_i64_i32", "v_div_scale")


def sregs(text: str) -> set[int]:
    out = set()
    for m in SREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def valu_sgpr_dest(ins: Insn) -> set[int]:
    """SGPRs a VALU instruction writes (readfirstlane / readlane / compares' first operand, carry-outs' second)."""
    mn = ins.mnem
    if not mn.startswith("v_") or mn.startswith("v_mfma"):
        return set()
    ops = [o.strip() for o in ins.ops.split(",")]
    if not ops:
        return set()
    if mn.startswith(("v_readfirstlane", "v_readlane")) or (mn.startswith("v_cmp") and mn.endswith("_e64")):
        return sregs(ops[0])
    if mn.startswith(SDST2) and len(ops) > 1:
        return sregs(ops[1])
    return set()


def check_sgpr_vmem(name, body, need=5):
    """(producer, consumer, need, got) for asm VMEM instructions reading a fresh VALU-written SGPR."""
    blocks, _ = build_blocks(body)
    findings = []
    for i, (_, insns) in enumerate(blocks):
        prev = []
        if i > 0:
            pb = blocks[i - 1][1]
            if pb and not (pb[-1].mnem.startswith("s_branch") or pb[-1].mnem == "s_endpgm"):
                prev = pb[-8:]
        seq = prev + list(insns)
        for c in range(len(prev), len(seq)):
            cons = seq[c]
            if not (cons.in_asm and is_vmem(cons.mnem)):
                continue
            reads = sregs(cons.ops)
            if not reads:
                continue
            waits = 0
            for prod in reversed(seq[max(0, c - 8):c]):
                if valu_sgpr_dest(prod) & reads and waits < need:
                    findings.append((prod, cons, need, waits))
                    break
                if prod.mnem.startswith("s_") and not prod.mnem.startswith(("s_nop", "s_waitcnt", "s_cmp")):
                    reads = reads - sregs(prod.ops.split(",")[0])  # a later scalar write supersedes
                    if not reads:
                        break
                if prod.mnem == "s_nop":
                    try:
                        waits += int(prod.ops.split()[0], 0) + 1
                    except ValueError:
                        waits += 1
                else:
                    waits += 1
                if waits >= need:
                    break
    return findings


# ------------------------------------------------------------------ shipped-library comparison

def code_objects(lib_path):
    data = open(lib_path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    pos, objs = 0, []
    while True:
        i = data.find(magic, pos)
        if i < 0:
            break
        ne, = struct.unpack_from("<Q", data, i + 24)
        off = i + 32
        for _ in range(ne):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tl].decode()
            off += tl
            if "gfx950" in triple and sz:
                objs.append(data[i + o:i + o + sz])
        pos = i + 1
    return objs


def disasm_mnemonics(lib_path, tmpdir):
    """{symbol: [list of mnemonic sequences, one per code object holding it]}"""
    objdump = "/opt/rocm/llvm/bin/llvm-objdump"
    out = defaultdict(list)
    for k, co in enumerate(code_objects(lib_path)):
        p = os.path.join(tmpdir, f"co{k}.elf")
        with open(p, "wb") as f:
            f.write(co)
        txt = subprocess.run([objdump, "-d", "--mcpu=gfx950", p], capture_output=True, text=True, check=True).stdout
        cur, seq = None, []
        for line in txt.splitlines():
            m = re.match(r"^[0-9a-f]+ <([^>]+)>:$", line)
            if m:
                if cur:
                    out[cur].append(seq)
                cur, seq = m.group(1), []
                continue
            if cur and line.startswith("\t"):
                mn = line.strip().split(None, 1)[0]
                if not mn.startswith("."):  # ("..." = objdump skipping zero padding)
                    seq.append(mn)
        if cur:
            out[cur].append(seq)
    return out


def norm(seq):
    """Mnemonics as both printers agree on them: no alignment nops, no encoding
    suffix (the disassembler spells v_permlane*_swap_b32 with _e32)."""
    return [re.sub(r"_e(32|64)$", "", m) for m in seq if m not in ("s_nop", "s_code_end", "RETIRED")]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--same-as", default="", help="shipped library whose code objects the ISA must equal")
    ap.add_argument("-q", action="store_true")
    args = ap.parse_args(argv)
    bad = 0
    total_loads = total_ret = nfunc = nws = 0
    asm_seqs = {}
    for path in args.files:
        try:
            funcs = parse_functions(path)
        except Exception as e:  # noqa: BLE001
            print(f"{path}: parse error: {e}", file=sys.stderr)
            return 2
        for name, body in funcs.items():
            nfunc += 1
            asm_seqs.setdefault(name, []).append(norm([x.mnem for k, x in body if k == "insn"]))
            try:
                findings, loads, rets = check_function(name, body)
            except ValueError as e:
                print(f"{path}: {name}: {e}", file=sys.stderr)
                return 2
            total_loads += loads
            total_ret += rets
            for prod, cons, need, got in (check_wait_states(name, body) + check_xdl_asm_reads(name, body) +
                                          check_sgpr_vmem(name, body)):
                bad += 1
                nws += 1
                print(f"WAITSTATE {os.path.basename(path)}:{cons.line} {name}: `{cons.text}` reads the result of "
                      f"`{prod.text}` (line {prod.line}) after {got} of its {need} wait states (asm side unpadded)")
            for ins, reg, info in findings:
                bad += 1
                what = f"v{reg}" if reg is not None else info[0]
                print(f"HAZARD {os.path.basename(path)}:{ins.line} {name}: `{ins.text}` touches {what} "
                      f"(untracked load at line {info[1]}, tag {info[0]})")
    if not args.q:
        print(f"audited {nfunc} functions in {len(args.files)} files: {total_loads} untracked asm register loads, "
              f"{total_ret} retiring waits, {bad - nws} hazards; {nws} asm wait-state hazards")
    if args.same_as:
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            dis = disasm_mnemonics(args.same_as, td)
        mism = 0
        for name, seqs in asm_seqs.items():
            if name not in dis:
                print(f"MISMATCH {name}: in the ISA files, not in {args.same_as}")
                mism += 1
                continue
            def same(d, s):  # (zero padding after a function decodes as v_cndmask_b32)
                d = norm(d)
                return d[:len(s)] == s and all(x == "v_cndmask_b32" for x in d[len(s):])
            for s in seqs:
                if not any(same(d, s) for d in dis[name]):
                    print(f"MISMATCH {name}: instruction sequence differs from the shipped code object")
                    mism += 1
        if not args.q:
            print(f"compared {len(asm_seqs)} functions with {args.same_as}: {mism} mismatches")
        bad += mism
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
