import re, sys
s=open(sys.argv[1]).read()
funcs=re.findall(r'^(_Z\S*):(?:\s*;.*)?$', s, re.M)
def regs(tok):
    m=re.match(r'v\[(\d+):(\d+)\]', tok)
    if m: return set(range(int(m.group(1)), int(m.group(2))+1))
    m=re.match(r'v(\d+)$', tok)
    if m: return {int(m.group(1))}
    return set()
for f in funcs:
    i=s.index('\n'+f+':'); j=s.index('.Lfunc_end',i)
    lines=s[i:j].split('\n')
    pending={}  # reg -> line idx of load
    hits=[]
    for k,l in enumerate(lines):
        t=l.strip()
        if not t or t.startswith(';') or t.startswith('.'): continue
        ops=[x.strip() for x in re.split(r'[ ,]+', t) if x.strip()]
        op=ops[0]
        if op.startswith('s_waitcnt') and 'vmcnt(0)' in t:
            pending.clear(); continue
        if op.startswith('buffer_load') and ' lds' not in t and 'offen' in t:
            for r in regs(ops[1]): pending[r]=k
            continue
        if op.startswith('v_mov') and len(ops)>=3:
            src=regs(ops[2])
            if src & set(pending):
                hits.append((k, t, min(pending[r] for r in src & set(pending))))
        # a write to a pending reg (not a load) ends tracking
        if op.startswith('v_') and len(ops)>=2:
            for r in regs(ops[1]): pending.pop(r, None)
    if hits:
        print(f, len(hits))
        for h in hits[:6]: print('   ', h)
