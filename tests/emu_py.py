"""ctypes view of tests/emu (host emulation of the kernels' fp32 arithmetic)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
EMU_DIR = os.path.join(HERE, "emu")
EMU_SO = os.path.join(EMU_DIR, "build", "libdcte_emu.so")
LUMA_SCALE = 1275000.0
# default_tie_tau(N) in dcte_capi.cpp: twice the derived error bound (test_tau_bound.py)
TIE_TAU = {2: 4e-6, 4: 4e-6, 8: 2e-5, 16: 5e-5}

_u8p = ctypes.POINTER(ctypes.c_uint8)
_f32p = ctypes.POINTER(ctypes.c_float)
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.run(["make", "-s", "-C", EMU_DIR], check=True)
        L = ctypes.CDLL(EMU_SO)
        L.emu_energy_map.restype = ctypes.c_int
        L.emu_energy_map.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                     ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     _f32p, _f32p, _f32p]
        L.emu_tau_search.restype = ctypes.c_double
        L.emu_tau_search.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_ulonglong, _u8p,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        L.emu_window_delta.restype = ctypes.c_double
        L.emu_window_delta.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p,
                                       ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def tau_search(n, sem=0, bpp=3, restarts=32, iters=2000, seed=1):
    """Adversarial search (tests/emu/tau_search.cpp) -> (delta, window, me, mt):
    the largest fp32 error of a candidate maximum, relative to the window's
    max coefficient, that the search found."""
    win = np.zeros((n, n, bpp) if bpp > 1 else (n, n), np.uint8)
    me, mt = ctypes.c_double(), ctypes.c_double()
    d = lib().emu_tau_search(n, sem, bpp, restarts, iters, seed, win.ctypes.data_as(_u8p),
                             ctypes.byref(me), ctypes.byref(mt))
    return d, win, me.value, mt.value


def window_delta(n, win, sem=0):
    win = np.ascontiguousarray(win, dtype=np.uint8)
    bpp = 1 if win.ndim == 2 else win.shape[2]
    me, mt = ctypes.c_double(), ctypes.c_double()
    d = lib().emu_window_delta(n, sem, bpp, win.ctypes.data_as(_u8p), ctypes.byref(me), ctypes.byref(mt))
    return d, me.value, mt.value


def scale(n, sem=0):
    return (LUMA_SCALE if sem == 0 else 1.0) * (n if n >= 8 else 1)


def kernel_weights(n, edges, textures, sem=0):
    """The launcher's pre-scaled weights (dcte_capi.cpp run_device)."""
    s = scale(n, sem)
    return np.float32(np.float64(np.float32(edges)) / s), np.float32(np.float64(np.float32(textures)) / s)


def energy_map(img, n, edges, textures, sem=0):
    """-> (E_fast, m_e, m_t), exactly the kernel's fast-path values
    (sem 0 = liblqr callback semantics, 1 = preview semantics)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    bpp = 1 if img.ndim == 2 else img.shape[2]
    we, wt = kernel_weights(n, edges, textures, sem)
    E = np.empty((h, w), np.float32)
    me = np.empty_like(E)
    mt = np.empty_like(E)
    rc = lib().emu_energy_map(img.ctypes.data_as(_u8p), w, h, bpp, w * bpp, n, we, wt, sem, 0, h,
                              E.ctypes.data_as(_f32p), me.ctypes.data_as(_f32p),
                              mt.ctypes.data_as(_f32p))
    assert rc == 0
    return E, me, mt


def refine_mask(me, mt, edges, textures, n, tau=None):
    """Pixels the kernel hands to the fp64 refinement (same predicate; tau
    defaults to the library's margin for N)."""
    if tau is None:
        tau = TIE_TAU[n]
    if np.float32(edges) == np.float32(textures):
        return np.zeros(me.shape, bool)
    hi = np.maximum(me, mt)
    lo = np.minimum(me, mt)
    return lo > (np.float32(1) - np.float32(tau)) * hi
