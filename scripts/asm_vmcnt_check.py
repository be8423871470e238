"""Static check of an asm-staged kernel's explicit vmcnt waits (diagnostics).

usage: python scripts/asm_vmcnt_check.py file.s SYMBOL_SUBSTRING
Walks the kernel's instructions in text order, running the loop that carries
the staging loads twice, and models the vector-memory counter: loads and
stores retire in issue order, `s_waitcnt vmcnt(N)` retires all but the
youngest N.  A hazard is an instruction that reads or writes a register of a
load that has not retired (the compiler does not track asm-issued loads).
Branches other than the loop back-edge are ignored (the paths that skip code
only issue fewer younger operations before a wait, i.e. wait longer)."""
import re
import sys


def regs(tok):
    m = re.match(r'^([va])\[(\d+):(\d+)\]$', tok)
    if m:
        return {f'{m.group(1)}{i}' for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r'^([va])(\d+)$', tok)
    return {tok} if m else set()


def main(path, sym):
    txt = open(path).read().split('\n')
    start = next(i for i, l in enumerate(txt) if re.match(r'^_Z\S*' + re.escape(sym) + r'\S*:', l))
    end = next(i for i in range(start, len(txt)) if txt[i].startswith('.Lfunc_end'))
    body = txt[start:end]
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r'^(\.LBB\S+):', l)] if m}
    # the loop with the most vector loads
    best = None
    for i, l in enumerate(body):
        m = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\S+)', l)
        if m and labels[m.group(1)] < i:
            a = labels[m.group(1)]
            nl = sum(1 for x in body[a:i] if x.strip().startswith('global_load'))
            if best is None or nl > best[2]:
                best = (a, i, nl)
    if best is None:
        print('no loop')
        return 1
    a, b, _ = best
    order = list(range(0, b + 1)) + list(range(a, b + 1)) + list(range(a, len(body)))
    pend = []  # (dest regs, text) in issue order
    bad = 0
    for i in order:
        l = body[i].strip()
        if not l or l.startswith(('.', ';')) or l.endswith(':'):
            continue
        op = l.split()[0]
        m = re.match(r's_waitcnt\s+.*vmcnt\((\d+)\)', l)
        if m:
            n = int(m.group(1))
            pend = pend[len(pend) - n:] if n < len(pend) else pend
            if n == 0:
                pend = []
            continue
        ops = [o.rstrip(',') for o in l.split()[1:]]
        touched = set().union(*[regs(o) for o in ops]) if ops else set()
        if op.startswith(('global_load', 'buffer_load')):
            # the address operands are read at issue: check them, then track the destination
            dst, srcs = regs(ops[0]), set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
            for r, t in pend:
                if r & (srcs | dst):
                    print('HAZARD', i, l, '<- in flight:', t)
                    bad += 1
            pend.append((dst, l))
            continue
        if op.startswith(('global_store', 'buffer_store', 'global_atomic')):
            for r, t in pend:
                if r & touched:
                    print('HAZARD', i, l, '<- in flight:', t)
                    bad += 1
            pend.append((set(), l))
            continue
        if op.startswith('s_') and not op.startswith('s_waitcnt'):
            continue
        for r, t in pend:
            if r & touched:
                print('HAZARD', i, l, '<- in flight:', t)
                bad += 1
                break
    print(f'loop {a}..{b}, {bad} hazards')
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1], sys.argv[2]))
