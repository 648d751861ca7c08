"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file.

    python tools/isa_blocks.py file.s KERNEL_SYMBOL [--min-mfma N]

Prints, for each block holding >= N MFMAs, the counts of MFMA / VALU / LDS / VMEM / SALU /
waitcnt / scratch instructions and the v_mov count (register shuffles)."""
import re
import sys
from collections import Counter


def blocks(path, sym):
    lines = open(path).read().split('\n')
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith('.Lfunc_end'))
    cur, name = [], 'entry'
    for l in lines[start + 1:end]:
        m = re.match(r'^(\.LBB\w+):', l)
        if m:
            yield name, cur
            cur, name = [], m.group(1)
            continue
        t = l.strip()
        if not t or t.startswith(';') or t.startswith('.'):
            continue
        cur.append(t.split()[0])
    yield name, cur


def classify(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('scratch_'):
        return 'scratch'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_')):
        return 'vmem'
    if op.startswith('s_waitcnt'):
        return 'wait'
    if op.startswith('s_barrier'):
        return 'barrier'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_'):
        return 'salu'
    return 'other'


def main():
    path, sym = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index('--min-mfma') + 1]) if '--min-mfma' in sys.argv else 1
    tot = Counter()
    for name, ops in blocks(path, sym):
        c = Counter(classify(o) for o in ops)
        tot.update(c)
        movs = sum(1 for o in ops if o.startswith(('v_mov', 'v_accvgpr')))
        trans = sum(1 for o in ops if o.startswith(('v_exp', 'v_log', 'v_rcp', 'v_sqrt', 'v_rsq', 'v_sin', 'v_cos')))
        if c['mfma'] >= mn:
            print(f"{name:14s} n={len(ops):5d} mfma={c['mfma']:3d} valu={c['valu']:4d} (mov {movs:3d}, trans {trans:3d}) "
                  f"lds={c['lds']:3d} vmem={c['vmem']:3d} salu={c['salu']:3d} wait={c['wait']:3d} "
                  f"bar={c['barrier']} scratch={c['scratch']}")
    print('total', dict(tot))


if __name__ == '__main__':
    main()
