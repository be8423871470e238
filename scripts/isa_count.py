"""Instruction-class histogram of one kernel's hot loop in a hipcc -S dump.

usage: python scripts/isa_count.py file.s SYMBOL_SUBSTRING
Prints the back-edges found and, for the largest loop body, counts of VALU /
readlane / MFMA / LDS / VMEM / SALU instructions (diagnostics only)."""
import collections
import re
import sys

txt = open(sys.argv[1]).read().split('\n')
start = next(i for i, l in enumerate(txt) if re.match(r'^_Z\S*' + re.escape(sys.argv[2]) + r'\S*:', l))
end = next(i for i in range(start, len(txt)) if txt[i].startswith('.Lfunc_end'))
body = txt[start:end]
labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
loops = []
for i, l in enumerate(body):
    m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\S+)', l)
    if m and labels[m.group(1)] < i:
        loops.append((labels[m.group(1)], i))
print('loops', loops)


def count(a, b):
    c = collections.Counter()
    for l in body[a:b]:
        l = l.strip()
        if not l or l.startswith(('.', ';')) or l.endswith(':'):
            continue
        op = l.split()[0]
        if op.startswith('v_mfma'):
            k = 'mfma'
        elif op.startswith(('v_readlane', 'v_readfirstlane', 'v_writelane')):
            k = 'readlane'
        elif op.startswith('v_'):
            k = 'valu'
            c['  ' + op] += 1
        elif op.startswith(('s_waitcnt', 's_nop')):
            k = 'wait/nop'
        elif op.startswith('s_'):
            k = 'salu'
        elif op.startswith('ds_'):
            k = 'lds'
        elif op.startswith(('global_', 'buffer_', 'scratch_')):
            k = 'vmem'
        else:
            k = 'other'
        c[k] += 1
    return c


a, b = max(loops, key=lambda t: t[1] - t[0])
print('loop lines', a, b)
for k, v in sorted(count(a, b).items(), key=lambda x: -x[1]):
    print(f'{v:5d} {k}')
