"""ctypes bindings to the CPU oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/build/libdcte_oracle.so (the C restatement of the reference's hot
path, oracle/dcte_oracle.c) and, where it was built, oracle/_ref/libdcte_ref.so
(the reference's own fft2d transforms, oracle/ref_harness.c).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "libdcte_oracle.so")
REF_SO = os.path.join(ORACLE_DIR, "_ref", "libdcte_ref.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)

_lib = None
_ref = None


def _ptr(a, t):
    return a.ctypes.data_as(t)


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            build_oracle()
        L = ctypes.CDLL(ORACLE_SO)
        L.orc_energy_map_rows.restype = ctypes.c_int
        L.orc_energy_map_rows.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, _f32p]
        L.orc_energy_map_luma_rows.restype = ctypes.c_int
        L.orc_energy_map_luma_rows.argtypes = [_f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                               ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, _f32p]
        L.orc_window_energy.restype = ctypes.c_float
        L.orc_window_energy.argtypes = [ctypes.c_int, _f64p, ctypes.c_float, ctypes.c_float]
        L.orc_dct.restype = ctypes.c_int
        L.orc_dct.argtypes = [ctypes.c_int, _f64p]
        L.orc_luma.restype = ctypes.c_double
        L.orc_luma.argtypes = [_u8p, ctypes.c_int]
        L.orc_max_threads.restype = ctypes.c_int
        L.orc_preview_luma.restype = ctypes.c_uint8
        L.orc_preview_luma.argtypes = [_u8p, ctypes.c_int]
        L.orc_preview_map_rows.restype = ctypes.c_int
        L.orc_preview_map_rows.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_size_t, ctypes.c_int, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, _f32p]
        L.orc_seam_find.restype = ctypes.c_int
        L.orc_seam_find.argtypes = [_f32p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_int), ctypes.c_void_p]
        _lib = L
    return _lib


def ref_available():
    return os.path.exists(REF_SO)


def ref():
    global _ref
    if _ref is None:
        if not ref_available():
            return None
        R = ctypes.CDLL(REF_SO)
        R.ref_energy_map_luma.restype = ctypes.c_int
        R.ref_energy_map_luma.argtypes = [_f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, ctypes.c_float, _f32p]
        R.ref_energy_map_luma_rows.restype = ctypes.c_int
        R.ref_energy_map_luma_rows.argtypes = [_f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                               ctypes.c_int, ctypes.c_int, _f32p]
        R.ref_window_energy.restype = ctypes.c_float
        R.ref_window_energy.argtypes = [ctypes.c_int, _f64p, ctypes.c_float, ctypes.c_float]
        R.ref_preview_map.restype = ctypes.c_int
        R.ref_preview_map.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_float, ctypes.c_float, _f32p]
        R.ref_dct.restype = ctypes.c_int
        R.ref_dct.argtypes = [ctypes.c_int, _f64p]
        _ref = R
    return _ref


# ---------------------------------------------------------------- oracle API
def energy_map(px, n, edges, textures, y0=0, y1=None, nthreads=1):
    """Energy map of an HxW (grey) or HxWx3 (RGB) uint8 image; rows [y0, y1)."""
    px = np.ascontiguousarray(px, dtype=np.uint8)
    h, w = px.shape[:2]
    bpp = 1 if px.ndim == 2 else px.shape[2]
    if y1 is None:
        y1 = h
    out = np.empty((y1 - y0, w), np.float32)
    rc = lib().orc_energy_map_rows(_ptr(px, _u8p), w, h, bpp, w * bpp, n,
                                   edges, textures, y0, y1, nthreads, _ptr(out, _f32p))
    if rc != 0:
        raise ValueError(f"oracle rejected the call (rc={rc})")
    return out


def energy_map_luma(luma, n, edges, textures, nthreads=1):
    luma = np.ascontiguousarray(luma, dtype=np.float64)
    h, w = luma.shape
    out = np.empty((h, w), np.float32)
    rc = lib().orc_energy_map_luma_rows(_ptr(luma, _f64p), 0, h, w, h, n, edges, textures,
                                        0, h, nthreads, _ptr(out, _f32p))
    if rc != 0:
        raise ValueError(f"oracle rejected the call (rc={rc})")
    return out


def preview_map(px, n, edges, textures, y0=0, y1=None, nthreads=1):
    """Preview-semantics energies (src/render.c:31-79) of an HxW / HxWxC region."""
    px = np.ascontiguousarray(px, dtype=np.uint8)
    h, w = px.shape[:2]
    bpp = 1 if px.ndim == 2 else px.shape[2]
    if y1 is None:
        y1 = h
    out = np.empty((y1 - y0, w), np.float32)
    rc = lib().orc_preview_map_rows(_ptr(px, _u8p), w, h, bpp, w * bpp, n, edges, textures,
                                    y0, y1, nthreads, _ptr(out, _f32p))
    if rc != 0:
        raise ValueError(f"oracle rejected the call (rc={rc})")
    return out


def seam_find(E, with_m=False):
    """liblqr-style minimum vertical seam of an HxW float32 energy map
    (delta_x 1, rigidity 0; leftmost minimum on ties) [liblqr, unverified]."""
    E = np.ascontiguousarray(E, dtype=np.float32)
    h, w = E.shape
    seam = np.empty(h, np.int32)
    M = np.empty((h, w), np.float32) if with_m else None
    rc = lib().orc_seam_find(_ptr(E, _f32p), w, w, h, seam.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                             M.ctypes.data if with_m else None)
    if rc != 0:
        raise ValueError("oracle rejected the map")
    return (seam, M) if with_m else seam


def window_energy(win, edges, textures):
    win = np.ascontiguousarray(win, dtype=np.float64)
    return float(lib().orc_window_energy(win.shape[0], _ptr(win, _f64p), edges, textures))


def dct(win):
    d = np.array(win, dtype=np.float64, order="C")
    rc = lib().orc_dct(d.shape[0], _ptr(d, _f64p))
    if rc != 0:
        raise ValueError("unsupported N")
    return d


def luma_plane(px):
    """liblqr LQR_ER_LUMA plane in double, exactly as the oracle computes it."""
    px = np.asarray(px, dtype=np.uint8)
    if px.ndim == 2:
        return px.astype(np.float64) / 255
    r = px[..., 0].astype(np.float64) / 255
    g = px[..., 1].astype(np.float64) / 255
    b = px[..., 2].astype(np.float64) / 255
    return 0.2126 * r + 0.7152 * g + 0.0722 * b


# ------------------------------------------------------------- reference API
def ref_energy_map_luma(luma, n, edges, textures):
    R = ref()
    luma = np.ascontiguousarray(luma, dtype=np.float64)
    h, w = luma.shape
    out = np.empty((h, w), np.float32)
    rc = R.ref_energy_map_luma(_ptr(luma, _f64p), w, h, n, edges, textures, _ptr(out, _f32p))
    if rc != 0:
        raise ValueError("reference rejected the call")
    return out


def ref_energy_map_luma_rows(luma, n, edges, textures, y0=0, y1=None, h=None, nthreads=1):
    """Rows [y0, y1) of the reference map of a luma plane whose first `h` rows
    are the frame (OpenMP over rows, one reference scratch per thread)."""
    R = ref()
    luma = np.ascontiguousarray(luma, dtype=np.float64)
    h = luma.shape[0] if h is None else h
    w = luma.shape[1]
    y1 = h if y1 is None else y1
    out = np.empty((y1 - y0, w), np.float32)
    rc = R.ref_energy_map_luma_rows(_ptr(luma, _f64p), w, h, n, edges, textures, y0, y1,
                                    nthreads, _ptr(out, _f32p))
    if rc != 0:
        raise ValueError("reference rejected the call")
    return out


def ref_preview_map(px, n, edges, textures):
    px = np.ascontiguousarray(px, dtype=np.uint8)
    h, w = px.shape[:2]
    bpp = 1 if px.ndim == 2 else px.shape[2]
    out = np.empty((h, w), np.float32)
    rc = ref().ref_preview_map(_ptr(px, _u8p), w, h, bpp, n, edges, textures, _ptr(out, _f32p))
    if rc != 0:
        raise ValueError("reference rejected the call")
    return out


def ref_window_energy(win, edges, textures):
    win = np.ascontiguousarray(win, dtype=np.float64)
    return float(ref().ref_window_energy(win.shape[0], _ptr(win, _f64p), edges, textures))


def ref_dct(win):
    d = np.array(win, dtype=np.float64, order="C")
    ref().ref_dct(d.shape[0], _ptr(d, _f64p))
    return d


# ------------------------------------------------------- u8 normalisation
def normalize_preview(E, channels=1, minmax=None):
    """normalize_image (src/render.c:81-109) + DOUBLE2GUCHAR (src/render.h:6) +
    GIMP ROUND ((int)(x + 0.5)), in double; max == min -> 0 (guarded).
    minmax: the whole frame's (min, max) when E is one band of it."""
    d = np.asarray(E, dtype=np.float32).astype(np.float64)
    mn, mx = (d.min(), d.max()) if minmax is None else (float(minmax[0]), float(minmax[1]))
    if not mx > mn:
        v = np.zeros(d.shape, np.uint8)
    else:
        v = (255 * ((d - mn) / (mx - mn)) + 0.5).astype(np.int32).astype(np.uint8)
    return np.repeat(v[..., None], channels, -1) if channels > 1 else v


def normalize_lqr(E, channels=1, minmax=None):
    """lqr_carver_get_energy_image as documented in include/dctenergy.h
    [liblqr, unverified]: (E - min)/(max - min) in float, x255, truncated.
    minmax: the whole frame's (min, max) when E is one band of it."""
    e = np.asarray(E, dtype=np.float32)
    mn, mx = (e.min(), e.max()) if minmax is None else (np.float32(minmax[0]), np.float32(minmax[1]))
    if not mx > mn:
        v = np.zeros(e.shape, np.uint8)
    else:
        v = (((e - mn) / (mx - mn)).astype(np.float32) * np.float32(255)).astype(np.int32).astype(np.uint8)
    return np.repeat(v[..., None], channels, -1) if channels > 1 else v
