"""Branch / wait / MFMA / LDS counts of every kernel in a hipcc -S dump whose
symbol contains one of the given substrings (diagnostics only).
usage: python scripts/isa_branches.py file.s SUBSTR [SUBSTR ...]"""
import collections
import re
import sys

txt = open(sys.argv[1]).read().split('\n')
for i, l in enumerate(txt):
    m = re.match(r'^(_Z\S+):', l)
    if not m or not any(s in m.group(1) for s in sys.argv[2:]):
        continue
    end = next(k for k in range(i, len(txt)) if txt[k].startswith('.Lfunc_end'))
    c = collections.Counter()
    for l2 in txt[i:end]:
        l2 = l2.strip()
        if not l2 or l2.startswith(('.', ';')) or l2.endswith(':'):
            continue
        op = l2.split()[0]
        c['branch' if op.startswith('s_cbranch') else 'waitcnt' if op == 's_waitcnt' else
          'mfma' if op.startswith('v_mfma') else 'ds' if op.startswith('ds_') else
          'vmem' if op.startswith(('global_', 'buffer_', 'flat_')) else 'other'] += 1
    print(f"{m.group(1)[:70]:70s} lines {end - i:6d} " + " ".join(f"{k} {c[k]}" for k in
                                                         ("branch", "waitcnt", "mfma", "ds", "vmem")))
