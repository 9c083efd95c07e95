"""LDS bank-conflict model of the batched-decode role form's accesses
(fattn_bdp.h, Q8_0 / Q4_0, D = 128; tools/lds_model.py rules): per access, the
cycles over its lane groups (1.0x = conflict-free) and, weighted by how often a
wave issues it per 64-key tile, the share of the kernel's LDS cycles it holds.
Verdict r04 item 6 (36 % of LDS-active cycles in bank conflicts)."""
import contextlib
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
with contextlib.redirect_stdout(io.StringIO()):
    import lds_model as M

lanes = range(64)
rows = []  # (name, cycles, groups, per-tile count over the workgroup)


def acc(name, addrs, width, kind="read", count=1):
    c, n = M.cost(addrs, width, kind)
    rows.append((name, c, n, count))


OLD = (lambda k: (k >> 3) & 1, lambda k: (k >> 2) & 3)           # fattn_bd.h / fattn_pf.h swizzles
NEW = (lambda k: ((k >> 2) ^ (k >> 3)) & 1, lambda k: (k >> 1) & 3)  # bdp_kswz / bdp_vswz (round 5)


def model(kt, RB, BB, swz=NEW, tag="new swizzles"):
    kswz, vswz = swz
    rows.clear()
    D, NK = 128, 8
    # build waves (4): per tile, per half-block (2 per wave) K and V: 5 qs dwords + the scale dword
    for hb in range(8):
        b, h = hb >> 1, hb & 1
        q0 = BB * b + 2 + (16 * h if kt == "q8_0" else 0)
        for j in range(5):
            acc(f"build raw qs dword (hb{hb} j{j})", [l * RB + (q0 & ~3) + 4 * j for l in lanes], 4, count=2)
        acc(f"build raw scale dword (hb{hb})", [l * RB + ((BB * b) & ~3) for l in lanes], 4, count=2)
    sk, sv = kswz, vswz
    for hb in range(8):
        b, h = hb >> 1, hb & 1
        for k in range(2):
            acc(f"build K image write (hb{hb} k{k})", [hb * 2048 + l * 32 + ((sk(l) ^ k) * 16) for l in lanes], 16,
                "write")
            acc(f"build V image write (hb{hb} k{k})", [4096 * 2 + b * 4096 + l * 64 + (((2 * h + k) ^ sv(l)) * 16)
                                                      for l in lanes], 16, "write")
    # compute waves (4): K operand reads (NK b128), V^T tr reads (2 x 2 x NDB b64 pairs), mask reads (4 b64)
    c32 = lambda l: l & 31
    hh = lambda l: l >> 5
    for kh in range(2):
        kbase = [kh * 1024 + c32(l) * 32 + ((hh(l) ^ kswz(c32(l))) * 16) for l in lanes]
        for kk in range(NK):
            acc(f"compute K read (kh{kh} kk{kk})", [x + kk * 2048 for x in kbase], 16, count=2)

    def vb(l, e, kh):
        gi, dh, h = l & 15, (l >> 4) & 1, l >> 5
        row = 8 * e + 4 * h + (gi >> 2)
        ch = (2 * dh + ((gi & 3) >> 1)) ^ vswz(row)
        return kh * 2048 + row * 64 + ch * 16 + (gi & 1) * 8
    for kh in range(2):
        for e in range(2):
            for q in range(2):
                for db in range(4):
                    acc(f"compute V^T tr read (kh{kh} e{e} q{q} db{db})", [vb(l, e, kh) + db * 4096 + q * 1024
                                                                         for l in lanes], 8, count=2)
    for u in range(4):
        acc(f"compute mask read (u{u})", [c32(l) * 16 + hh(l) * 8 + u * 512 for l in lanes], 8, count=4)
    tot = sum(c * k for _, c, _, k in rows)
    ideal = sum(n * k for _, _, n, k in rows)
    print(f"== fattn_bdp_kernel {kt} ({tag}), D = 128, raw rows of {RB} B: LDS cycles per 64-key tile (workgroup) "
          f"{tot:.0f}, conflict-free {ideal:.0f}, in conflicts {(tot - ideal) / tot:.1%}")
    groups = {}
    for name, c, n, k in rows:
        key = name.split(" (")[0]
        g = groups.setdefault(key, [0, 0])
        g[0] += c * k
        g[1] += n * k
    for key, (c, n) in sorted(groups.items(), key=lambda kv: -(kv[1][0] - kv[1][1])):
        print(f"  {key:28s} cycles {c:7.0f}  ideal {n:7.0f}  ({c / n:.2f}x)  excess share {(c - n) / max(tot - ideal, 1):.1%}")


if __name__ == "__main__":
    model("q8_0", 136, 34, OLD, "round-4 swizzles")
    model("q8_0", 136, 34)
    model("q4_0", 72, 18)
