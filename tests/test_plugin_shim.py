"""Drop-in check: the patched liblqr callback, driven by a fake
liblqr energy build (tests/fake_lqr), served from libdctenergy_hip.so.

CPU: without a device the plug-in glue reports the error and every callback
runs the original per-window code -- the map equals the reference exactly.
GPU: at the carver's original size every callback is answered from the GPU
map (no per-window work) within the parity tolerance; once seams change the
carver size the original code takes over again.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import dctenergy
import oracle_py as O
from golden_util import load_input, within_tol

HERE = os.path.dirname(os.path.abspath(__file__))
FAKE_DIR = os.path.join(HERE, "fake_lqr")
_lib = None


def fake():
    global _lib
    if _lib is None:
        dctenergy.lib()
        O.lib()
        subprocess.run(["make", "-s", "-C", FAKE_DIR], check=True)
        L = ctypes.CDLL(os.path.join(FAKE_DIR, "build", "libfake_lqr.so"))
        L.fake_build_emap.restype = ctypes.c_int
        L.fake_build_emap.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                      ctypes.POINTER(ctypes.c_longlong),
                                      ctypes.POINTER(ctypes.c_int)]
        _lib = L
    return _lib


def build_emap(img, n, e, t, use_gpu, removed=0, transposed=False):
    img = np.ascontiguousarray(img)
    h, w = img.shape[:2]
    bpp = 1 if img.ndim == 2 else img.shape[2]
    out = np.empty((w - removed, h) if transposed else (h, w - removed), np.float32)
    calls = ctypes.c_longlong()
    status = ctypes.c_int()
    rc = fake().fake_build_emap(img.ctypes.data, w, h, bpp, n, e, t, int(use_gpu), removed,
                                int(transposed), out.ctypes.data, ctypes.byref(calls),
                                ctypes.byref(status))
    assert rc == 0
    return out, calls.value, status.value


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_original_path_without_gpu(n):
    if dctenergy.device_count() > 0:
        pytest.skip("device visible; covered by the GPU test")
    img = load_input("natural_rgb_73x59.npy")
    out, calls, status = build_emap(img, n, 0.15, 0.85, use_gpu=True)
    assert status == dctenergy.DCTE_ENODEV
    assert calls == img.shape[0] * img.shape[1]
    assert np.array_equal(out, O.energy_map(img, n, 0.15, 0.85))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_gpu_map_serves_callbacks(n):
    img = load_input("natural_rgb_97x41.npy")
    out, calls, status = build_emap(img, n, 0.15, 0.85, use_gpu=True)
    assert status == dctenergy.DCTE_OK
    assert calls == 0
    assert within_tol(out, O.energy_map(img, n, 0.15, 0.85)).all()
    # after 3 "seams": carver is narrower -> original code, exact
    out2, calls2, _ = build_emap(img, n, 0.15, 0.85, use_gpu=True, removed=3)
    assert calls2 == img.shape[0] * (img.shape[1] - 3)
    assert np.array_equal(out2, O.energy_map(np.ascontiguousarray(img[:, :-3]), n, 0.15, 0.85))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 8, 16])
def test_gpu_map_serves_transposed_carver(n):
    """Vertical resize: liblqr evaluates the energy on the transposed carver;
    the transposed map answers those callbacks."""
    img = load_input("natural_rgb_73x59.npy")
    out, calls, status = build_emap(img, n, 0.15, 0.85, use_gpu=True, transposed=True)
    assert status == dctenergy.DCTE_OK
    assert calls == 0
    ref = O.energy_map(np.ascontiguousarray(np.swapaxes(img, 0, 1)), n, 0.15, 0.85)
    assert within_tol(out, ref).all()
