"""Instruction-mix summary of a gfx950 .s file (hipcc --save-temps).

    python tools/isa_stats.py dcte_kernels-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]
"""
import re
import sys
from collections import Counter


def main():
    s = open(sys.argv[1]).read()
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r'^(_Z\S*):\s*;', s, re.M):
        name = m.group(1)
        if filt not in name:
            continue
        end = s.index('.Lfunc_end', m.end())
        body = s[m.end():end]
        ins = [l.strip() for l in body.split('\n')
               if l.startswith('\t') and l.strip() and not l.strip().startswith(('.', ';'))]
        c = Counter(i.split()[0] for i in ins)
        valu = sum(v for k, v in c.items() if k.startswith('v_'))
        print(f"{name[:44]:44s} total {len(ins):5d} valu {valu:5d} fma {c.get('v_fma_f32', 0):4d} "
              f"max3 {c.get('v_max3_f32', 0):4d} pk {sum(v for k, v in c.items() if k.startswith('v_pk')):3d} "
              f"ds_rd {sum(v for k, v in c.items() if k.startswith('ds_read')):4d} "
              f"ds_wr {sum(v for k, v in c.items() if k.startswith('ds_write')):3d} "
              f"bar {c.get('s_barrier', 0)} scratch {sum(v for k, v in c.items() if 'scratch' in k)} "
              f"vmcnt0 {body.count('vmcnt(0)')}")
        if len(sys.argv) > 3:
            for k, v in c.most_common(40):
                print('   ', k, v)


if __name__ == '__main__':
    main()
