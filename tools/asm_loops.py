"""Largest basic blocks of one kernel in a hipcc -S listing: instruction mix per block.
usage: python tools/asm_loops.py <file.s> <mangled-name-substring> [min_instructions]"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 200
start = [i for i, l in enumerate(lines) if re.match(r'^_Z\S*' + re.escape(key) + r'\S*:', l)][0]
end = [j for j in range(start, len(lines)) if lines[j].strip().startswith('.Lfunc_end')][0]
body = lines[start:end]
blocks, cur = [], None
for l in body:
    t = l.strip()
    if re.match(r'^\.LBB\d+_\d+:', t):
        cur = [t, Counter()]
        blocks.append(cur)
        continue
    if cur is None or not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    cur[1][t.split()[0]] += 1
for name, c in blocks:
    n = sum(c.values())
    if n < mn:
        continue
    valu = sum(v for k, v in c.items() if k.startswith('v_'))
    ld = sum(v for k, v in c.items() if 'load' in k and not k.startswith('s_'))
    st = sum(v for k, v in c.items() if 'store' in k)
    print(f"{name} n={n} valu={valu} vmem_ld={ld} vmem_st={st} top={c.most_common(12)}")
