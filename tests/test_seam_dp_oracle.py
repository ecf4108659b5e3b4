"""CPU: the seam-DP restatement (oracle/dcte_oracle.c orc_seam_find) against
an independent numpy statement of the same recursion and, on tiny maps,
against exhaustive search over every 8-connected seam.  [liblqr, unverified:
liblqr is not in this image; the recursion follows the carver configuration
lqr_carver_init(carver, 1, 0) at src/render.c:313.]"""
import itertools

import numpy as np
import pytest

import oracle_py as O


def numpy_seam(E):
    h, w = E.shape
    M = E[0].copy()
    par = np.zeros((h, w), np.int64)
    for y in range(1, h):
        inf = np.float32(np.inf)
        left = np.concatenate([[inf], M[:-1]])
        right = np.concatenate([M[1:], [inf]])
        cand = np.stack([left, M, right])           # leftmost first
        k = np.argmin(cand, 0)                      # argmin keeps the first minimum
        par[y] = k - 1
        M = (E[y] + cand[k, np.arange(w)]).astype(np.float32)
    x = int(np.argmin(M))
    seam = [x]
    for y in range(h - 1, 0, -1):
        x += int(par[y, x])
        seam.append(x)
    return np.array(seam[::-1], np.int32), M


@pytest.mark.parametrize("shape", [(1, 1), (1, 7), (9, 1), (2, 2), (17, 33), (64, 40), (130, 257)])
@pytest.mark.parametrize("kind", ["uniform", "ties", "ramp"])
def test_oracle_matches_numpy(shape, kind):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1] + 7 * len(kind))
    h, w = shape
    if kind == "uniform":
        E = rng.random((h, w), dtype=np.float32)
    elif kind == "ties":
        E = rng.integers(0, 3, (h, w)).astype(np.float32)
    else:
        E = np.tile(np.abs(np.arange(w) - w / 3).astype(np.float32), (h, 1))
    seam, M = O.seam_find(E, with_m=True)
    ref, Mlast = numpy_seam(E)
    assert np.array_equal(seam, ref)
    assert np.array_equal(M[-1], Mlast)
    assert (np.abs(np.diff(seam)) <= 1).all()


@pytest.mark.parametrize("seed", range(6))
def test_oracle_seam_is_a_minimum(seed):
    rng = np.random.default_rng(seed)
    h, w = 5, 4
    E = rng.integers(0, 4, (h, w)).astype(np.float32)
    seam = O.seam_find(E)
    best = min(sum(E[y, s[y]] for y in range(h))
               for s in itertools.product(range(w), repeat=h)
               if all(abs(s[y + 1] - s[y]) <= 1 for y in range(h - 1)))
    assert sum(E[y, seam[y]] for y in range(h)) == best
