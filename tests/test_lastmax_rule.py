"""The refinement kernels decide the class with maxima instead of the
reference's index-tracking scan (dcte_kernels.hip lastmax_decide /
lastmax_group).  This checks the rule against the scan itself
(src/dct.c:100-109: max <= currval keeps the LAST maximum over the non-DC
coefficients; edge atoms (0,1) and (1,0), src/dct.c:18-25) on coefficient
arrays built to tie: repeated maxima at random positions, edge/texture ties,
all-zero windows.  CPU only."""
import numpy as np
import pytest


def scan(C):
    n = C.shape[0]
    m, b1, b2 = 0.0, 0, 0
    for k1 in range(n):
        for k2 in range(n):
            v = abs(C[k1, k2])
            if m <= v and (k1 or k2):
                m, b1, b2 = v, k1, k2
    return m, (b1, b2) in ((0, 1), (1, 0))


def rule(C):
    """lastmax_decide over the flat index order k1 * N + k2."""
    n = C.shape[0]
    a = np.abs(C.reshape(-1))
    a01, a10 = a[1], a[n]
    mb = a[2:n].max() if n > 2 else -1.0
    ma = a[n + 1:].max()
    m = max(ma, a10, mb, a01)
    return m, (not ma == m) and (a10 == m or ((not mb == m) and a01 == m))


def group_rule(C):
    """lastmax_group: row k1 = l per lane, the group reduction, lane 0 decides."""
    n = C.shape[0]
    rows = np.abs(C)
    pa = []
    for l in range(n):
        v = rows[l]
        mb_l = v[2:].max() if n > 2 else -1.0
        p = max(mb_l, v[1])
        pa.append(max(p, v[0]) if l >= 2 else (p if l == 1 else -1.0))
    ma = max(pa)
    mb = rows[0, 2:].max() if n > 2 else -1.0
    m = max(ma, rows[1, 0], mb, rows[0, 1])
    return m, (not ma == m) and (rows[1, 0] == m or ((not mb == m) and rows[0, 1] == m))


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_rule_equals_scan(n):
    rng = np.random.default_rng(n)
    for trial in range(4000):
        C = rng.normal(size=(n, n)) * (rng.random() < 0.9)
        k = rng.integers(0, 4)
        if k:   # plant ties of the maximum at random places, signs random
            top = np.abs(C).max() + rng.random()
            for idx in rng.choice(n * n, size=min(n * n, 1 + rng.integers(0, 4)), replace=False):
                C.flat[idx] = top * rng.choice([-1, 1])
        if trial % 7 == 0:   # edge / texture tie at the top
            top = np.abs(C).max() + 1
            C[0, 1] = top
            C.flat[rng.integers(2, n * n)] = -top if n > 1 else top
        if trial % 11 == 0:
            C[1, 0] = np.abs(C).max() + 1
            C[0, 1] = -C[1, 0]
        if trial % 13 == 0:
            C[:] = 0.0
        assert rule(C) == scan(C), (C, rule(C), scan(C))
        assert group_rule(C) == scan(C), (C, group_rule(C), scan(C))
