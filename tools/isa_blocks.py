"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file (diagnostic).
Usage: python tools/isa_blocks.py file.s kernel_substring [min_instructions]"""
import collections
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    L = open(path).read().split('\n')
    s = next(i for i, l in enumerate(L) if re.match(r'^_Z\S*:', l) and key in l)
    e = next(i for i in range(s, len(L)) if 's_endpgm' in L[i])
    blocks, cur = [], None
    for i in range(s, e + 1):
        l = L[i]
        if i == s or re.match(r'^\.LBB\d+_\d+:', l):
            cur = [l.split(':')[0][:20], i, []]
            blocks.append(cur)
        elif l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;'):
            cur[2].append(l.strip())
    tot = collections.Counter()
    for name, i, ins in blocks:
        c = collections.Counter()
        for x in ins:
            op = x.split()[0]
            if op.startswith('v_mfma'): k = 'mfma'
            elif op.startswith(('v_exp', 'v_log', 'v_rcp', 'v_rsq', 'v_sqrt')): k = 'trans'
            elif op.startswith('ds_'): k = 'ds'
            elif op.startswith('scratch_'): k = 'SCRATCH'
            elif op.startswith(('global_', 'buffer_')): k = 'vmem'
            elif op.startswith('v_accvgpr'): k = 'accmov'
            elif op.startswith('v_'): k = 'valu'
            elif op.startswith('s_waitcnt'): k = 'wait'
            elif op.startswith('s_barrier'): k = 'barrier'
            elif op.startswith('s_'): k = 'salu'
            else: k = 'other'
            c[k] += 1
        tot.update(c)
        if len(ins) >= mn:
            print(f"{name:20s} line {i:6d} n={len(ins):5d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
    print("total", dict(tot))


if __name__ == '__main__':
    main()
