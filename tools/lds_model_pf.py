"""LDS bank-conflict model of the prefill kernel's accesses (tools/lds_model.py rules):
which of its LDS reads and writes conflict, and by how much."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import io, contextlib
with contextlib.redirect_stdout(io.StringIO()):
    import lds_model as M
lanes = range(64)
print("== pf kernel (Q8_0, D=128, 64-key tiles)")
# K image reads b128: kbase + kk*2048 + t*1024
for t in range(2):
    M.show(f"K img read t{t}", [(l & 31) * 32 + (((l >> 5) ^ (((l & 31) >> 3) & 1)) * 16) + t * 1024 for l in lanes], 16)
# V tr reads (8 B per lane), per e
for e in range(2):
    def va(l, e=e):
        gi = l & 15; dh = (l >> 4) & 1; h = l >> 5
        row = 8 * e + 4 * h + (gi >> 2)
        ch = (2 * dh + ((gi & 3) >> 1)) ^ ((h + 2 * e) & 3)
        return row * 64 + ch * 16 + (gi & 1) * 8
    M.show(f"V tr read e{e}", [va(l) for l in lanes], 8)
# mask reads b64: (c32*8 + ((4t+u) ^ ((c32>>1)&7)))*16 + 8h
for t in range(2):
    for u in range(4):
        M.show(f"mask read t{t} u{u}", [((l & 31) * 8 + ((4 * t + u) ^ (((l & 31) >> 1) & 7))) * 16 + 8 * (l >> 5) for l in lanes], 8)
# dequant raw reads: row = lane, 5 dwords from qb, 136-B rows
for b in range(4):
    for h in range(2):
        q0 = 34 * b + 2 + 16 * h
        for j in range(5):
            M.show(f"raw read b{b} h{h} dw{j}", [l * 136 + (q0 & ~3) + 4 * j for l in lanes], 4)
        M.show(f"raw scale b{b}", [l * 136 + ((34 * b) & ~3) for l in lanes], 4)
# dequant image writes b128: K kd = w*2048 + lane*32 + sk*16 ; V vd = b*4096 + lane*64 + chunk
M.show("K img write", [l * 32 + (((l >> 3) & 1) * 16) for l in lanes], 16, "write")
for h in range(2):
    M.show(f"V img write h{h}", [l * 64 + (((2 * h) ^ ((l >> 2) & 3)) * 16) for l in lanes], 16, "write")
