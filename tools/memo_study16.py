"""CPU study: could a per-wave window memo serve the N = 16 dense walk?
(r04; no GPU.)  Line art (tools/fix_study.py frame, 2048^2 crop): the flagged
windows of dense strips in the flat walk's order, 16-pixel batches; (1) a
32-slot direct-mapped table per chunk of C consecutive batches never holds a
whole batch (16 distinct keys collide); (2) a fully associative 32-entry LRU,
even over the whole frame, answers 26 % of windows and 1.4 % of batches --
the frame's distinct flagged windows outnumber what 9 KB of LDS holds (260 B
each).  So no N = 16 memo.

    python tools/memo_study16.py
"""
import sys, numpy as np, hashlib
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tools'), os.path.join(ROOT, 'dct-carver_amd')]
import memo_study as M, torch
from fix_study import frames
S=2048; n=16
fr=frames(S, torch, "cpu")
img=fr["lineart_grey"].numpy()
entries=[]   # flat list: dense strips (> 32 flags) in strip order, entries row-major
for ty in range(0,S,64):   # N=16 tile_h? use 64 rows
    win=M.windows(img,n,ty,min(S,ty+64)); f=M.flags(win.astype(np.float64),4e-6)
    for sx in range(0,S,64):
        ys,xs=np.nonzero(f[:,sx:sx+64])
        if len(ys)<=32: continue
        entries += [win[y,sx+x].tobytes() for y,x in zip(ys,xs)]
nb=(len(entries)+15)//16
print("entries",len(entries),"batches",nb)
slot=lambda k: int.from_bytes(hashlib.blake2b(k,digest_size=4).digest(),'little')%32
for C in (4, 8, 16, 32, 64):
    full=0; tot=0
    for c0 in range(0,nb,C):   # one wave per chunk of C batches
        tab={}
        for b in range(c0,min(nb,c0+C)):
            batch=entries[16*b:16*b+16]
            allhit=all(tab.get(slot(k))==k for k in batch)
            full+=allhit; tot+=1
            if not allhit:
                for k in batch: tab[slot(k)]=k
    print("C",C,"all-hit batches",round(full/tot,3))
from collections import OrderedDict
for E in (32,):
  for C in (8,16,32,64,1<<30):
    full=0; tot=0; whit=0
    for c0 in range(0,nb,C):
        tab=OrderedDict()
        for b in range(c0,min(nb,c0+C)):
            batch=entries[16*b:16*b+16]
            hits=[k in tab for k in batch]; whit+=sum(hits)
            allhit=all(hits); full+=allhit; tot+=1
            for k in batch:
                if k in tab: tab.move_to_end(k)
                else:
                    tab[k]=1
                    if len(tab)>E: tab.popitem(last=False)
    print("assoc",E,"C",C,"all-hit",round(full/tot,3),"window hit",round(whit/len(entries),3))
