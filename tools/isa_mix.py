"""Instruction mix per basic block of selected kernels in a hipcc -save-temps .s (dev tool)."""
import re
import sys
from collections import Counter


def cat(o):
    if o.startswith('v_'):
        return 'valu'
    if o.startswith('s_'):
        return 'salu'
    if o.startswith('ds_'):
        return 'lds'
    if o.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    return 'other'


path, pat = sys.argv[1], sys.argv[2]
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 50
s = open(path).read()
for m in re.finditer(r'\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end', s, re.S):
    name, body = m.group(1), m.group(2)
    if pat not in name:
        continue
    print('==', name)
    blocks = re.split(r'\n(?=\.LBB\d+_\d+:)', body)
    tot = Counter()
    for b in blocks:
        lab = b.split(':')[0] if b.startswith('.LBB') else 'entry'
        ops = [l.strip().split()[0] for l in b.split('\n') if l.startswith('\t') and not l.strip().startswith(('.', ';'))]
        c = Counter(cat(o) for o in ops)
        tot.update(c)
        if len(ops) >= minlen:
            det = Counter(ops).most_common(12)
            print(f'  {lab:12s} n={len(ops):5d} {dict(c)}')
            print('      ', det)
    print('  total', dict(tot))
    vg = re.search(r'\.vgpr_count:\s+(\d+)', s[m.end():])
