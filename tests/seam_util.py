"""Seam helpers for the seam-update tests (numpy; test infrastructure)."""
import numpy as np


def halo(n, sem):
    hl = n // 2 - 1 if sem == 0 else (n - 1) // 2 - 1
    return hl, n - 1 - hl


def carve(img, seam):
    """Remove pixel seam[y] from every row y."""
    h, w = img.shape[:2]
    keep = np.ones((h, w), bool)
    keep[np.arange(h), seam] = False
    return np.ascontiguousarray(img[keep].reshape((h, w - 1) + img.shape[2:]))


def seam_span(seam, w, n, sem):
    """Per row: min / max of the seam over the window rows (clamped)."""
    h = len(seam)
    hl, hr = halo(n, sem)
    rows = np.clip(np.arange(h)[:, None] + np.arange(-hl, hr + 1)[None, :], 0, h - 1)
    s = np.clip(np.asarray(seam), 0, w - 1)[rows]
    return s.min(1), s.max(1), hl, hr


def random_seams(h, w, seed, count):
    """8-connected random walks, plus seams that jump and hug the borders."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        kind = k % 4
        if kind == 0:      # connected walk
            s = np.empty(h, np.int64)
            s[0] = rng.integers(0, w)
            for y in range(1, h):
                s[y] = np.clip(s[y - 1] + rng.integers(-1, 2), 0, w - 1)
        elif kind == 1:    # arbitrary per-row positions
            s = rng.integers(0, w, h)
        elif kind == 2:    # left border
            s = np.clip(rng.integers(-1, 3, h), 0, w - 1)
        else:              # right border
            s = np.clip(w - 1 - rng.integers(0, 3, h), 0, w - 1)
        out.append(s.astype(np.int32))
    return out
