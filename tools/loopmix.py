#!/usr/bin/env python3
"""Instruction mix of a kernel's loops in a -save-temps ISA file (diagnostic):
python tools/loopmix.py build/isa/fattn_launch_d128.s <mangled-kernel-name-prefix>"""
import collections
import sys


def main(path, name):
    L = open(path).read().split('\n')
    start = [i for i, l in enumerate(L) if l.startswith(name) and l.split(':')[0].startswith(name)][0]
    end = [i for i in range(start, len(L)) if 's_endpgm' in L[i]][0]
    body = L[start:end]
    for h, l in enumerate(body):
        if 'Loop Header' not in l:
            continue
        lab = (body[h] if body[h].startswith('.LBB') else body[h - 1]).split(':')[0]
        be = [i for i, x in enumerate(body) if ('s_cbranch' in x or 's_branch' in x) and x.split()[-1] == lab]
        if not be:
            continue
        seg = body[h:max(be) + 1]
        c = collections.Counter(x.strip().split()[0] for x in seg
                                if x.strip() and not x.strip().startswith((';', '.')))
        mf = sum(v for k, v in c.items() if k.startswith('v_mfma'))
        valu = sum(v for k, v in c.items() if k.startswith('v_') and not k.startswith('v_mfma'))
        print(f"loop {lab}: mfma {mf} valu {valu} lds {sum(v for k, v in c.items() if k.startswith('ds_'))} "
              f"salu {sum(v for k, v in c.items() if k.startswith('s_'))}")
        print("  ", c.most_common(16))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
