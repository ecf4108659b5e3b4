"""The context-free CPU entries of SURVEY §8b (dcte_energy_window,
dcte_normalize_u8_host): plain host code in libdctenergy_hip.so, no device.

Pinned bit-exactly to the golden fixtures generated from the reference's own
transforms (tests/golden/make_golden.py): every KAT window, and every preview
map's u8 layer (normalize_image, src/render.c:81-109).
"""
import numpy as np
import pytest

import dctenergy
import oracle_py as O
from golden_util import load_kat, load_map, manifest


def test_energy_window_matches_every_kat():
    for k in manifest()["kat"]:
        win = load_kat(k["window"])
        got = dctenergy.energy_window(win, k["edges"], k["textures"])
        assert got == np.float32(k["energy"]), k


def test_energy_window_bit_exact_vs_oracle_random():
    rng = np.random.default_rng(7)
    for n in (2, 4, 8, 16):
        for scale in (1e-4, 1.0, 300.0):
            for _ in range(200):
                w = rng.standard_normal((n, n)) * scale
                e, t = rng.random(2).astype(np.float32)
                assert dctenergy.energy_window(w, e, t) == O.window_energy(w, e, t)


def test_energy_window_ties_and_window_untouched():
    # exact edge/texture ties: the last maximum decides (src/dct.c:103)
    for n in (2, 4, 8, 16):
        k = np.arange(n)
        a01 = np.outer(np.ones(n), np.cos(np.pi * (k + 0.5) / n))
        a11 = np.outer(np.cos(np.pi * (k + 0.5) / n), np.cos(np.pi * (k + 0.5) / n))
        for w in (a01, a01 + a11, np.full((n, n), 0.3), np.zeros((n, n))):
            w0 = w.copy()
            assert dctenergy.energy_window(w, 0.2, 0.9) == O.window_energy(w0, 0.2, 0.9)
            assert np.array_equal(w, w0)


def test_energy_window_rejects_bad_n():
    for n in (1, 3, 6, 32):
        with pytest.raises(dctenergy.DcteError):
            dctenergy.energy_window(np.zeros((n, n)), 0.5, 0.5)


@pytest.mark.parametrize("entry", manifest()["preview"], ids=lambda e: e["output_u8"])
def test_normalize_u8_host_matches_golden_preview_layer(entry):
    E = load_map(entry["output"])
    got = dctenergy.normalize_u8_host(E, dctenergy.DCTE_NORM_PREVIEW, entry["channels"])
    assert np.array_equal(got, load_map(entry["output_u8"]))


def test_normalize_u8_host_lqr_mode_and_flat():
    rng = np.random.default_rng(3)
    E = rng.random((33, 17), dtype=np.float32) * 5
    mn, mx = E.min(), E.max()
    want = ((E - mn) / (mx - mn) * np.float32(255)).astype(np.int32).astype(np.uint8)
    assert np.array_equal(dctenergy.normalize_u8_host(E, dctenergy.DCTE_NORM_LQR), want)
    # max == min: 0 (the reference divides by zero there, src/render.c:101)
    flat = np.full((4, 5), 2.5, np.float32)
    assert not dctenergy.normalize_u8_host(flat, dctenergy.DCTE_NORM_PREVIEW, 3).any()
    with pytest.raises(dctenergy.DcteError):
        dctenergy.normalize_u8_host(E, 7)
