"""Print instruction mix of every loop (backward branch) in one kernel of a
hipcc -S output: python tools/asm_loops.py file.s kernel_symbol"""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.index(name + ':')
j = s.index('.Lfunc_end', i)
body = s[i:j].splitlines()
labels = {l.split(':')[0]: k for k, l in enumerate(body) if l.startswith('.LBB')}
for k, l in enumerate(body):
    t = l.strip()
    if t.startswith('s_cbranch') or t.startswith('s_branch'):
        tgt = t.split()[-1]
        if tgt in labels and labels[tgt] < k:
            seg = body[labels[tgt]:k + 1]
            c = Counter(x.strip().split()[0] for x in seg
                        if x.strip() and not x.strip().startswith(('.', ';')) and ':' not in x.split()[0])
            v = sum(n for op, n in c.items() if op.startswith('v_') and 'mfma' not in op)
            m = sum(n for op, n in c.items() if 'mfma' in op)
            print(f'loop {tgt} lines {k - labels[tgt]} valu {v} mfma {m}')
            print('   ', [(op, n) for op, n in c.most_common(60)])
