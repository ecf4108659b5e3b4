"""The refinement margin tau: a DERIVED bound, checked against an adversarial
search (CPU only).

The kernel refines a pixel in fp64 when its fp32 maxima m_e and m_t lie
within tau of each other (dcte_capi.cpp default_tie_tau(N), dcte_kernels.hip
emit): lo > (1 - tau) hi.  An unrefined pixel keeps the reference's class as
long as
    tau - 2u >= (delta_e + delta_t) (1 + delta),     u = 2^-24,
delta_x = max over windows of |m_x(fp32) - m_x(reference)| / M (M = the
window's largest non-DC coefficient).  tests/emu/tau_bound.cpp DERIVES the
delta's from the kernels' own operation sequence (dcte_passes.h /
dcte_math.h compiled over a tracking type on a symbolic window): fp32
rounding (forward error analysis relative to M), the fp32 constants, and
the reference's own error against exact arithmetic -- its fp64 transform in
its operation order (dcte_ref64.h tracked the same way) and liblqr's double
luma against the integer luma.  The tests demand tau_N >= 2x the derived
requirement, and that the adversarial search (tests/emu/tau_search.cpp: hill
climbing over integer windows with the kernel's fp32 code against the exact
transform) never finds more than the derived fp32 bound -- a check of the
derivation itself.
Reference arithmetic: src/fft2d/shrtdct.c:61-117, 238-386,
src/fft2d/fftsg2d.c:566-627, decision src/dct.c:100-109.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import emu_py as EM
import oracle_py as O
from golden_util import ATOL, RTOL

U32 = 2.0 ** -24
LUMA_ULP = 5 * 2.0 ** -53 * 1275000   # liblqr's double luma vs the integer luma, per sample (L units)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def derived(n, sem=0):
    """-> dict of the derived terms for N, semantics (relative to M)."""
    L = EM.lib()
    L.tau_bound.restype = ctypes.c_int
    L.tau_bound.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    L.tau_ref_error.restype = ctypes.c_double
    L.tau_ref_error.argtypes = [ctypes.c_int, ctypes.c_double]
    out = np.zeros(13)
    xmax = 637500.0 if sem == 0 else 128.0        # |biased luma| (dcte_luma.h)
    rc = L.tau_bound(n, xmax, out.ctypes.data)
    assert rc == 0, (n, sem, out.tolist())
    m_min = out[7]                               # hat units of the integer luma
    # the reference's units: orthonormal (hat / N) for N = 8, 16; unnormalised N = 2, 4;
    # liblqr luma = L / 1275000, the preview's u8 luma as is
    unit = (n if n >= 8 else 1) * (1275000.0 if sem == 0 else 1.0)
    ref64 = L.tau_ref_error(n, 1.0 if sem == 0 else 255.0)
    assert ref64 >= 0
    rho64 = ref64 / (m_min / unit)
    rho_luma = out[4] * LUMA_ULP / m_min if sem == 0 else 0.0
    d = {"fp32_e": out[0], "fp32_t": out[1], "const_e": out[2], "const_t": out[3],
         "ref64": rho64, "ref_luma": rho_luma, "l1_e": out[10], "l1_t": out[11],
         "events": int(out[12]), "cands_t": int(out[6])}
    d["delta_e"] = d["fp32_e"] + d["const_e"] + rho64 + rho_luma
    d["delta_t"] = d["fp32_t"] + d["const_t"] + rho64 + rho_luma
    d["need"] = (d["delta_e"] + d["delta_t"]) * (1 + max(d["delta_e"], d["delta_t"])) + 2 * U32
    return d


@pytest.mark.parametrize("sem", [0, 1])
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_tau_covers_twice_the_derived_bound(n, sem):
    """The library's margin for N is at least twice what the derivation
    requires; the derivation covers every coefficient of both classes (its
    candidate sets are exactly the reference's atoms) and never rounds a
    brightness-carrying value."""
    d = derived(n, sem)
    assert d["cands_t"] == n * n - 3
    tau = EM.TIE_TAU[n]
    assert tau - 2 * U32 >= 2 * (d["need"] - 2 * U32), (n, sem, tau, d)
    print(n, sem, json.dumps({k: (float(f"{v:.4g}") if isinstance(v, float) else v) for k, v in d.items()}))


def test_tau_table_matches_the_library():
    """EM.TIE_TAU mirrors dcte_capi.cpp's default_tie_tau."""
    src = open(os.path.join(ROOT, "dct-carver_amd", "csrc", "dcte_capi.cpp")).read()
    assert "double default_tie_tau(int n) { return n == 16 ? 5e-5 : n == 8 ? 2e-5 : 4e-6; }" in src
    assert EM.TIE_TAU == {2: 4e-6, 4: 4e-6, 8: 2e-5, 16: 5e-5}


@pytest.mark.parametrize("sem", [0, 1])
@pytest.mark.parametrize("bpp", [1, 3])
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_search_stays_below_the_derived_bound(n, bpp, sem):
    """The adversarial search's worst window (the kernel's fp32 code against
    the exact transform in long double) stays under the derived fp32 bound:
    the derivation is not contradicted by any window found."""
    restarts, iters = (24, 1500) if n == 16 else (64, 2000)
    d, win, me, mt = EM.tau_search(n, sem, bpp, restarts, iters, seed=100 + n + 10 * bpp + sem)
    b = derived(n, sem)
    assert 0 <= d <= max(b["fp32_e"] + b["const_e"], b["fp32_t"] + b["const_t"]), (n, bpp, sem, d, b)
    assert d <= EM.TIE_TAU[n] / 4
    # the window found is an ordinary input: as a frame, its own pixel (HL, HL)
    # -- no clamping -- is within tolerance of the oracle or handed to the fp64 pass
    hl = n // 2 - 1 if sem == 0 else (n - 1) // 2 - 1
    if sem == 0:
        ref = O.energy_map(win, n, 0.3, 0.7)[hl, hl]
    else:
        ref = O.preview_map(win, n, 0.3, 0.7)[hl, hl]
    E, me32, mt32 = EM.energy_map(win, n, 0.3, 0.7, sem=sem)
    refined = EM.refine_mask(me32, mt32, 0.3, 0.7, n)[hl, hl]
    assert refined or abs(float(E[hl, hl]) - float(ref)) <= RTOL * abs(float(ref)) + ATOL


def test_committed_long_searches_below_the_derived_bound():
    """The committed long searches (up to 15 M windows per case) stay under
    the derived fp32 bound and reproduce from their stored windows."""
    base = os.path.join(ROOT, "profiles", "r05")
    rows = [json.loads(l) for l in open(os.path.join(base, "tau_search.jsonl"))]
    rows += [json.loads(l) for l in open(os.path.join(base, "tau_search_n16_long.jsonl"))]
    assert {r["n"] for r in rows} == {2, 4, 8, 16}
    bounds = {}
    for r in rows:
        key = (r["n"], r["sem"])
        if key not in bounds:
            b = derived(*key)
            bounds[key] = max(b["fp32_e"] + b["const_e"], b["fp32_t"] + b["const_t"])
        assert r["delta"] <= bounds[key], r
        d, _, _ = EM.window_delta(r["n"], np.array(r["window"], np.uint8), r["sem"])
        assert abs(d - r["delta"]) <= 1e-12, r           # reproducible from the stored window
