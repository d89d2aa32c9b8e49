#!/usr/bin/env python3
"""Instruction mix per loop of one kernel in an amdgcn .s file (dev tool).
usage: loopmix.py file.s symbol-substring"""
import collections, re, sys
L = open(sys.argv[1]).read().split('\n')
s = [i for i, l in enumerate(L) if re.match(r'^_Z\S*:', l) and sys.argv[2] in l.split(':')[0]][0]
e = [i for i in range(s, len(L)) if L[i].startswith('.Lfunc_end')][0]
loops, order = {}, []
cur = None
for i in range(s, e):
    m2 = re.match(r'^(\.LBB\d+_\d+):', L[i]) or re.match(r'^; %bb', L[i])
    if m2:
        m = re.search(r'Loop: Header=(\S+) Depth=(\d)', L[i])
        cur = (m.group(1), m.group(2)) if m else ('top', '0')
        if cur not in loops: order.append(cur)
    t = L[i].strip()
    if L[i].startswith('\t') and t and not t.startswith(';') and not t.startswith('.'):
        loops.setdefault(cur, []).append(t.split()[0] + (' dpp' if 'quad_perm' in t or 'row_' in t else ''))
for k in order:
    v = loops.get(k, [])
    c = collections.Counter()
    for ins in v:
        if ins.startswith('v_'): c['valu'] += 1
        if ins.startswith('v_') and 'f64' in ins: c['f64'] += 1
        if ins.startswith('s_'): c['salu'] += 1
        if ins.startswith('ds_'): c['lds'] += 1
        if ins.startswith(('global_', 'buffer_', 'flat_')): c['vmem'] += 1
        if 'dpp' in ins or 'permlane' in ins: c['xlane'] += 1
        if 'waitcnt' in ins: c['wait'] += 1
    print(k, len(v), dict(c))
