"""libdctenergy_hip.so builds, loads and exports every symbol include/dctenergy.h
declares; argument validation and error codes work without a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import dctenergy

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dctenergy.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dcte_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = dctenergy.lib()
    names = declared_functions()
    assert len(names) >= 10
    for name in names:
        assert hasattr(L, name), name
    assert sorted(dctenergy.EXPORTS) == names


def test_abi_version_and_strerror():
    L = dctenergy.lib()
    assert L.dcte_abi_version() == 2
    for code in (0, -1, -2, -3, -4, -5, -6):
        assert L.dcte_strerror(code)
    assert L.dcte_strerror(-99) == b"unknown error"


def test_null_and_bad_arguments():
    L = dctenergy.lib()
    assert L.dcte_create(None, 1, 0) == dctenergy.DCTE_EINVAL
    assert L.dcte_set_option(None, 1, 0.0) == dctenergy.DCTE_EINVAL
    out = np.zeros((4, 4), np.float32)
    px = np.zeros((4, 4), np.uint8)
    assert L.dcte_energy_map(None, px.ctypes.data, 4, 4, 1, 4, 8, 0.5, 0.5, 0, 0,
                             out.ctypes.data) == dctenergy.DCTE_EINVAL
    L.dcte_destroy(None)  # no-op
    assert L.dcte_last_refined(None) == 0
    assert L.dcte_last_error(None) == b""


def test_no_device_is_an_error_not_a_fallback():
    """Without a GPU the product refuses to run (no silent CPU path)."""
    if dctenergy.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(dctenergy.DcteError) as ei:
        dctenergy.Context()
    assert ei.value.code == dctenergy.DCTE_ENODEV


def test_library_is_gfx950_code_object():
    """The shared object carries a gfx950 code object (the kernels)."""
    data = open(dctenergy.LIB_PATH, "rb").read()
    assert b"gfx950" in data
