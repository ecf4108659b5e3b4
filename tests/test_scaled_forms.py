"""The second (column) pass of the map kernel on its own, against float64.

The kernel folds every column transform's magnitudes into running maxima in
SCALED form (dcte_math.h dct8_col_sc / dct8_k0_sc / dct16_odd_sc, the N = 4
Cols): rotations by fixed angles are one FMA per output and the constant they
share is applied once per pixel.  This checks the pass -- compiled from the
kernel's own headers by tests/emu -- on random rings of row-transform outputs
against the plain transform in float64 (hat units, DCTE_HD docs in
dcte_math.h): m_e = the edge atoms C01 / C10, m_t = every other non-DC
coefficient (src/dct.c:96-110).  CPU only.
"""
import ctypes
import os

import numpy as np
import pytest

EMU_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "emu", "build", "libdcte_emu.so")


def _lib():
    if not os.path.exists(EMU_SO):
        pytest.skip("tests/emu not built (python __graft_entry__.py)")
    L = ctypes.CDLL(EMU_SO)
    fp = ctypes.POINTER(ctypes.c_float)
    L.emu_cols.argtypes = [ctypes.c_int, fp, ctypes.c_int, fp, fp]
    return L


def _hat(n):
    """Column transform in the kernel's hat units: X0 = sum, Xk = g * sum cos."""
    g = np.sqrt(2.0) if n >= 8 else 1.0
    j = np.arange(n)
    T = g * np.cos(np.pi * (2 * j[None, :] + 1) * np.arange(n)[:, None] / (2 * n))
    T[0] = 1.0
    return T


def _cols(L, n, ring, q=0):
    mt, me = ctypes.c_float(), ctypes.c_float()
    r = np.ascontiguousarray(ring, dtype=np.float32)
    assert L.emu_cols(n, r.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), q,
                      ctypes.byref(mt), ctypes.byref(me)) == 0
    return mt.value, me.value


def _rings(n, ch, rng, count=300):
    for i in range(count):
        ring = rng.normal(0, 10 ** rng.uniform(-2, 4), (n, ch))
        if i % 3 == 0:                       # channel 0: exact integer row sums
            ring[:, 0] = rng.integers(-5_000_000, 5_000_000, n)
        if i % 7 == 0:                       # a near-constant column
            ring[:, rng.integers(ch)] = 1234.5
        yield ring.astype(np.float32)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_column_pass_small_n(n):
    L = _lib()
    T = _hat(n)
    rng = np.random.default_rng(n)
    for ring in _rings(n, n, rng):
        C = np.abs(T @ ring.astype(np.float64))        # C[k2, k1]
        me_r = max(C[1, 0], C[0, 1])
        C[0, 0] = C[1, 0] = C[0, 1] = 0.0
        mt_r = C.max()
        mt, me = _cols(L, n, ring)
        m = max(mt_r, me_r, 1e-30)
        assert abs(mt - mt_r) <= 2e-6 * m, (mt, mt_r)
        assert abs(me - me_r) <= 2e-6 * m, (me, me_r)


@pytest.mark.parametrize("q", [0, 1, 2, 3])
def test_column_pass_n16(q):
    """N = 16: wave q's four channels; wave 0 channel 0 is k1 = 0 (C01 edge,
    DC excluded), wave 2 channel 0 is k1 = 1 (C10 edge)."""
    L = _lib()
    T = _hat(16)
    rng = np.random.default_rng(16 + q)
    for ring in _rings(16, 4, rng):
        C = np.abs(T @ ring.astype(np.float64))        # C[k2, c]
        me_r = 0.0
        if q == 0:
            me_r = C[1, 0]
            C[0, 0] = C[1, 0] = 0.0
        elif q == 2:
            me_r = C[0, 0]
            C[0, 0] = 0.0
        mt_r = C.max()
        mt, me = _cols(L, 16, ring, q)
        m = max(mt_r, me_r, 1e-30)
        assert abs(mt - mt_r) <= 2e-6 * m, (q, mt, mt_r)
        assert abs(me - me_r) <= 2e-6 * m, (q, me, me_r)
