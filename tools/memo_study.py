"""How often do the windows the refinement recomputes repeat?  (CPU study for
a window-memo in the dense refinement walks; no GPU.)

For each tie-dense frame of tools/fix_study.py (a crop of side --size), the
liblqr N x N windows whose fp64 edge and texture maxima lie within tau of each
other (the pixels the map kernel flags) are keyed by their exact bytes.
Reported per frame: flagged pixels, distinct windows over the frame, and the
fraction of flagged windows that an earlier flagged window of the SAME strip
(64 columns x --tile-h rows, the unit one refinement wave walks) already
carries -- the best a per-wave memo could skip -- and with a table of at most
--entries windows per strip (direct-mapped on a hash).

    python tools/memo_study.py [--size 2048] [--n 8]
"""
import argparse
import json
import os
import sys

import numpy as np
from scipy.fft import dctn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "dct-carver_amd")]


def windows(img, n, y0, y1):
    """(y1 - y0) x W x n x n windows (liblqr gather, clamped)"""
    h, w = img.shape
    hl = n // 2 - 1
    ys = np.clip(np.arange(y0, y1)[:, None] + np.arange(-hl, n - hl)[None, :], 0, h - 1)
    xs = np.clip(np.arange(w)[:, None] + np.arange(-hl, n - hl)[None, :], 0, w - 1)
    return img[ys[:, None, :, None], xs[None, :, None, :]]


def flags(win, tau):
    c = np.abs(dctn(win.astype(np.float64), type=2, norm="ortho", axes=(-2, -1)))
    me = np.maximum(c[..., 0, 1], c[..., 1, 0])
    c[..., 0, 0] = c[..., 0, 1] = c[..., 1, 0] = 0
    mt = c.max(axis=(-2, -1))
    hi = np.maximum(me, mt)
    return (np.abs(me - mt) <= tau * hi) & (hi > 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--tile-h", type=int, default=128)
    ap.add_argument("--entries", type=int, default=64)
    ap.add_argument("--tau", type=float, default=4e-6)
    a = ap.parse_args()
    import torch
    from fix_study import frames
    S, n = a.size, a.n
    fr = frames(S, torch, "cpu")
    for name in ("lineart_grey", "lineart_color", "grid8_grey", "dots64_grey", "text4_grey"):
        img = fr[name].numpy()
        lum = img
        if img.ndim == 3:   # colour: flags from the luma, keys on the three channels packed
            lum = img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114
            img = (img[..., 0].astype(np.uint32) << 16) | (img[..., 1].astype(np.uint32) << 8) | img[..., 2]
        nflag = 0
        seen_all = set()
        hit_strip = hit_tab = 0
        for ty in range(0, S, a.tile_h):
            win = windows(img, n, ty, min(S, ty + a.tile_h))
            f = flags(windows(lum, n, ty, min(S, ty + a.tile_h)), a.tau)
            for sx in range(0, S, 64):
                ys, xs = np.nonzero(f[:, sx:sx + 64])      # row-major: the list order
                seen, tab = set(), {}
                for y, x in zip(ys, xs):
                    k = win[y, sx + x].tobytes()
                    seen_all.add(k)
                    if k in seen:
                        hit_strip += 1
                    seen.add(k)
                    slot = hash(k) % a.entries
                    if tab.get(slot) == k:
                        hit_tab += 1
                    else:
                        tab[slot] = k
                nflag += len(ys)
        print(json.dumps({"frame": name, "size": S, "n": n, "flagged": nflag,
                          "distinct_windows": len(seen_all),
                          "strip_repeat_frac": round(hit_strip / max(nflag, 1), 4),
                          "table_hit_frac": round(hit_tab / max(nflag, 1), 4),
                          "entries": a.entries}), flush=True)


if __name__ == "__main__":
    main()
