"""The refinement margin tau against an adversarial search (CPU only).

The kernel refines a pixel in fp64 when its fp32 maxima m_e and m_t lie
within tau of each other (dcte_capi.cpp kDefaultTieTau, dcte_kernels.hip
emit); the class is only safe if no candidate's fp32 error exceeds tau/2 of
the window's max coefficient.  tests/emu/tau_search.cpp hill-climbs over
integer pixel windows (random restarts of six window kinds) for the largest
    delta = max(|m_e32 - m_e|, |m_t32 - m_t|) / max(m_e, m_t)
with the map kernel's own fp32 code against the exact transform, and this
test demands delta <= tau/4 (2x margin on top of the tau/2 requirement).
The long searches (1.5-20 M windows per case, tools/tau_long.py) are in
profiles/r05/tau_search.jsonl (re-run in r05 after the N = 16 odd half
moved to a scaled form; N = 2, 4, 8 reproduce r02's exactly) and, 7.5x
longer for N = 16, in profiles/r05/tau_search_n16_long.jsonl; the worst found
is 7.7e-7 = tau/5.2 (N = 16 grey; r04's N = 16 arithmetic at the same budget:
7.5e-7, tau_search_n16_long_r04arith.jsonl).
Reference arithmetic: src/fft2d/shrtdct.c:61-117, 238-386,
src/fft2d/fftsg2d.c:566-627, decision src/dct.c:100-109.
"""
import numpy as np
import pytest

import emu_py as EM
import oracle_py as O
from golden_util import ATOL, RTOL


@pytest.mark.parametrize("sem", [0, 1])
@pytest.mark.parametrize("bpp", [1, 3])
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_search_stays_below_quarter_tau(n, bpp, sem):
    restarts, iters = (24, 1500) if n == 16 else (64, 2000)
    d, win, me, mt = EM.tau_search(n, sem, bpp, restarts, iters, seed=100 + n + 10 * bpp + sem)
    assert 0 <= d <= EM.TIE_TAU / 4, (n, bpp, sem, d, win.tolist())
    # the window found is an ordinary input: as a frame, its own pixel (HL, HL)
    # -- no clamping -- is within tolerance of the oracle or handed to the fp64 pass
    hl = n // 2 - 1 if sem == 0 else (n - 1) // 2 - 1
    if sem == 0:
        ref = O.energy_map(win, n, 0.3, 0.7)[hl, hl]
    else:
        ref = O.preview_map(win, n, 0.3, 0.7)[hl, hl]
    E, me32, mt32 = EM.energy_map(win, n, 0.3, 0.7, sem=sem)
    refined = EM.refine_mask(me32, mt32, 0.3, 0.7)[hl, hl]
    assert refined or abs(float(E[hl, hl]) - float(ref)) <= RTOL * abs(float(ref)) + ATOL


def test_committed_long_search_margin():
    """The committed long searches all stay within tau/4."""
    import json
    import os
    base = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r05")
    rows = [json.loads(l) for l in open(os.path.join(base, "tau_search.jsonl"))]
    # plus r05's 7.5x longer N = 16 searches (15 M windows per case, six seeds)
    rows += [json.loads(l) for l in open(os.path.join(base, "tau_search_n16_long.jsonl"))]
    assert {r["n"] for r in rows} == {2, 4, 8, 16}
    for r in rows:
        assert r["delta"] <= EM.TIE_TAU / 4, r
        d, _, _ = EM.window_delta(r["n"], np.array(r["window"], np.uint8), r["sem"])
        assert abs(d - r["delta"]) <= 1e-12, r           # reproducible from the stored window
