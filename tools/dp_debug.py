import sys, numpy as np
sys.path[:0]=['dct-carver_amd','tests']
import dctenergy, oracle_py as O
from test_seam_dp import _maps, SHAPES
def run(ctx, E, tag):
    got=ctx.seam_find(E); ref=O.seam_find(E)
    ok=np.array_equal(got,ref)
    bad=np.nonzero(got!=ref)[0]
    print(tag, E.shape, ok, 'nbad', len(bad), 'rows', bad[:3], bad[-3:] if len(bad) else '', 'got', got[bad[:3]] if len(bad) else '', 'ref', ref[bad[:3]] if len(bad) else '', flush=True)
    return ok
with dctenergy.Context(ngpus=1) as ctx:
    for shape in SHAPES[:8]:
        for kind in ["uniform", "ties", "flat", "valley"]:
            h, w = shape
            run(ctx, _maps(h, w, kind, h * 7 + w), kind)
print("--- repeat flat 257x300 x3 then ties then flat")
with dctenergy.Context(ngpus=1) as ctx:
    for kind in ["flat","flat","flat","ties","flat","uniform","flat"]:
        run(ctx, _maps(257, 300, kind, 257 * 7 + 300), kind)
