"""Instruction mix per basic block of one kernel in a hipcc -S listing (the blocks with MFMAs
are the loop bodies).  usage: loop_mix.py file.s symbol_substring"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split('\n')
sym = [l for l in lines if l.startswith('_Z') and sys.argv[2] in l.split(':')[0] and ':' in l][0]
start = lines.index(sym)
end = [i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end')][0]
blocks, cur, name = [], [], 'entry'
for l in (x.strip() for x in lines[start:end]):
    if re.match(r'^\.LBB\d+_\d+:', l):
        blocks.append((name, cur))
        name, cur = l, []
    elif l and not l.startswith(('.', ';', '//')):
        cur.append(l)
blocks.append((name, cur))


def kind(op):
    if 'mfma' in op:
        return 'mfma'
    if op.startswith(('v_exp', 'v_rcp', 'v_log', 'v_sqrt', 'v_rsq')):
        return 'trans'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_')):
        return 'vmem'
    return op


for n, b in blocks:
    if len(b) < 20:
        continue
    print(n, len(b), dict(Counter(kind(x.split()[0]) for x in b)))
big = max(blocks, key=lambda nb: sum(1 for x in nb[1] if 'mfma' in x))
print('largest MFMA block', big[0])
print(Counter(x.split()[0] for x in big[1] if x.startswith('v_') and 'mfma' not in x).most_common(30))
