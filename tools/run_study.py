"""Would a sliding fp64 walk beat the per-window dense walks?  (VERDICT r04,
item 1's follow-up question.)  The exact map shares ddct8x8s / ddct16x16s
pass 1 (along the image row) between vertically adjacent pixels, so a
refinement walk could do the same for the flagged pixels of one column that
follow each other down a strip.  This measures how much there is to share:
the flagged set of the fp32 map (tests/emu's bit-exact host emulation of the
kernel, flag = the kernel's tau test at the default tau) on the tie-dense
frames of tools/fix_study.py, its vertical runs per column inside 128-row
tiles, and the transform count of a walk that keeps a ring alive across gaps
shorter than N - 1 rows (cost = rows covered + N column transforms per
flagged pixel) against 2 N transforms per window today.

    python tools/run_study.py [N] [S]      (needs tests/emu built: make -C tests/emu)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAU = 4e-6   # kDefaultTieTau, dcte_capi.cpp


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "emu", "build", "libdcte_emu.so"))
    yy, xx = np.mgrid[0:S, 0:S]
    rng = np.random.default_rng(5)
    blk = rng.random((S // 4 + 1, S // 4 + 1)) < 0.3
    kinds = {
        "lineart": np.where((yy % 23 == 0) | (xx % 31 == 0) | ((xx + 2 * yy) % 97 == 0), 0, 255),
        "grid8": np.where((yy % 8 == 0) | (xx % 8 == 0), 0, 255),
        "dots": np.where(rng.random((S, S)) < 1 / 64, 255, 16),
        "text": np.where(blk.repeat(4, 0).repeat(4, 1)[:S, :S], 0, 255),
    }
    keep = np.float32(1 - TAU)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    for name, g in kinds.items():
        px = np.ascontiguousarray(g.astype(np.uint8))
        E = np.empty((S, S), np.float32)
        me, mt = np.empty_like(E), np.empty_like(E)
        lib.emu_energy_map(P(px), S, S, 1, ctypes.c_size_t(S), n, ctypes.c_float(0.3),
                           ctypes.c_float(0.7), 0, 0, S, P(E), P(me), P(mt))
        f = (me > keep * mt) & (mt > keep * me)
        tot = int(f.sum())
        runs, rows, segs = [], 0, 0
        for t0 in range(0, S, 128):
            tile = f[t0:t0 + 128]
            for c in range(S):
                ys = np.nonzero(tile[:, c])[0]
                if len(ys) == 0:
                    continue
                d = np.diff(np.concatenate([[0], tile[:, c].astype(np.int8), [0]]))
                runs += list(np.nonzero(d == -1)[0] - np.nonzero(d == 1)[0])
                start = prev = ys[0]
                for y in ys[1:]:
                    if y - prev > n - 1:
                        rows += prev - start + n
                        segs += 1
                        start = y
                    prev = y
                rows += prev - start + n
                segs += 1
        runs = np.array(runs)
        print({"frame": name, "n": n, "size": S, "flagged_frac": round(tot / S / S, 4),
               "runs": len(runs), "mean_run": round(float(runs.mean()), 2) if len(runs) else 0,
               "px_per_ring_segment": round(tot / max(1, segs), 2),
               "transforms_vs_per_window": round((rows + n * tot) / (2 * n * max(1, tot)), 3)})


if __name__ == "__main__":
    main()
