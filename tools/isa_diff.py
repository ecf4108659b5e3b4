"""Per-kernel instruction-mix diff of two gfx950 .s files (hipcc --save-temps).

    python tools/isa_diff.py BEFORE.s AFTER.s [--rename 'from=>to' ...]

Kernels are matched by demangled name (after the --rename substitutions,
applied to BEFORE's names); for each, the full opcode histogram is compared.
Prints one line per kernel: identical / differs (with the opcode deltas) /
only in one file.
"""
import argparse
import re
import subprocess
from collections import Counter


def kernels(path):
    s = open(path).read()
    out = {}
    for m in re.finditer(r'^(_Z\S*):\s*;', s, re.M):
        name = m.group(1)
        end = s.index('.Lfunc_end', m.end())
        body = s[m.end():end]
        ins = [l.strip() for l in body.split('\n')
               if l.startswith('\t') and l.strip() and not l.strip().startswith(('.', ';'))]
        out[name] = Counter(i.split()[0] for i in ins)
    names = list(out)
    dem = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True, text=True).stdout.split('\n')
    return {d: out[n] for n, d in zip(names, dem)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('before')
    ap.add_argument('after')
    ap.add_argument('--rename', action='append', default=[])
    a = ap.parse_args()
    b, c = kernels(a.before), kernels(a.after)
    ren = [r.split('=>') for r in a.rename]
    bb = {}
    for k, v in b.items():
        for f, t in ren:
            k = k.replace(f, t)
        bb[k] = v
    for k in sorted(set(bb) | set(c)):
        if k not in c:
            print(f'removed    {k}  ({sum(bb[k].values())} insts)')
        elif k not in bb:
            print(f'new        {k}  ({sum(c[k].values())} insts)')
        elif bb[k] == c[k]:
            print(f'identical  {k}  ({sum(c[k].values())} insts)')
        else:
            d = {op: c[k][op] - bb[k][op] for op in set(bb[k]) | set(c[k]) if c[k][op] != bb[k][op]}
            print(f'differs    {k}  {sum(bb[k].values())} -> {sum(c[k].values())}: {d}')


if __name__ == '__main__':
    main()
