"""Per-loop-depth instruction census of one kernel in a hipcc -S listing (gfx950).

usage: python tools/isa_loops.py avr.s <mangled-kernel-name> [depth]
Counts VALU / SALU / VMEM / LDS / scratch / branch instructions in the basic blocks the
compiler annotates as belonging to loops of the given depth (default: the deepest)."""
import re
import sys
from collections import Counter


def blocks(lines):
    cur, depth, out = None, 0, []
    for l in lines:
        m = re.match(r'^(\.LBB\S+|; %bb\.\d+):', l.strip())
        if m or l.startswith('.LBB'):
            if cur is not None:
                out.append((depth, cur))
            cur = []
            d = re.search(r'Depth=(\d+)', l)
            depth = int(d.group(1)) if d else 0
            continue
        if cur is None:
            cur = []
        s = l.strip()
        if not s or s.startswith(';') or s.startswith('.'):
            d = re.search(r'Depth=(\d+)', s)
            if d and not cur:
                depth = int(d.group(1))
            continue
        cur.append(s.split()[0])
    if cur is not None:
        out.append((depth, cur))
    return out


def kind(op):
    if op.startswith('scratch_'):
        return 'scratch'
    if op.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('s_cbranch', 's_branch')):
        return 'branch'
    if op.startswith('s_waitcnt') or op.startswith('s_nop'):
        return 'wait/nop'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('v_mov'):
        return 'v_mov'
    if op.startswith('v_') and '_f64' in op:
        return 'valu_f64'
    if op.startswith('v_'):
        return 'valu'
    return 'other'


def main():
    text = open(sys.argv[1]).read()
    name = sys.argv[2]
    i = text.index(name + ':')
    j = text.index('.Lfunc_end', i)
    bl = blocks(text[i:j].split('\n'))
    maxd = max(d for d, _ in bl)
    want = int(sys.argv[3]) if len(sys.argv) > 3 else maxd
    tot = Counter()
    nb = 0
    for d, ops in bl:
        if d >= want:
            nb += 1
            for op in ops:
                tot[kind(op)] += 1
    allc = Counter(kind(op) for _, ops in bl for op in ops)
    print(f"depth>={want} (max {maxd}): {nb} blocks, {sum(tot.values())} instrs: {dict(tot)}")
    print(f"whole kernel: {sum(allc.values())} instrs: {dict(allc)}")


if __name__ == '__main__':
    main()
